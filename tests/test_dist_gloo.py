"""N>1 path on CPU: LPT sharding + record all-gather across 2 gloo ranks (no GPU)."""
import os
import random
import socket
import struct

import pytest
import torch.multiprocessing as mp

import sdz_dist


def test_lpt_shard_balances_and_covers():
    rng = random.Random(5)
    sizes = [int(4096 * 2 ** rng.uniform(0, 12)) for _ in range(1000)]
    for world in (1, 2, 3, 8):
        shards = sdz_dist.lpt_shard(sizes, world)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(sizes)))
        loads = [sum(sizes[i] for i in s) for s in shards]
        assert max(loads) - min(loads) <= max(sizes)       # LPT bound


def test_lpt_shard_deterministic_for_equal_sizes():
    assert sdz_dist.lpt_shard([7] * 8, 2) == [[0, 2, 4, 6], [1, 3, 5, 7]]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sizes, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shards = sdz_dist.lpt_shard(sizes, world)
    # each rank "decodes" its shard: a 64-byte record per stream (status, out_len, index)
    recs = b"".join(struct.pack("<iiQ", 0, rank, sizes[i] * 3) + struct.pack("<Q", i) + bytes(40)
                    for i in shards[rank])
    allrec = sdz_dist.gather_records(recs, 64, shards, rank)
    dist.destroy_process_group()
    q.put((rank, [struct.unpack("<iiQQ", r[:24]) for r in allrec]))


@pytest.mark.timeout(120)
def test_gather_records_world2_gloo():
    sizes = [100, 5, 70, 70, 1, 300, 2, 9]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    shards = sdz_dist.lpt_shard(sizes, 2)
    owner = {i: r for r, s in enumerate(shards) for i in s}
    for rank in (0, 1):
        got = res[rank]
        assert len(got) == len(sizes)
        for i, (st, rk, olen, idx) in enumerate(got):
            assert (st, rk, olen, idx) == (0, owner[i], sizes[i] * 3, i)
