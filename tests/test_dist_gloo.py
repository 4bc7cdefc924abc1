"""N>1 path: LPT sharding (libsdz's sdz_lpt_shard and the Python mirror agree) and the
record all-gather across 2 gloo ranks on CPU; and, on the GPU box, 2 ranks that each run the
real engine on their LPT shard of a C4-shaped batch and gather the records."""
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


def test_lpt_shard_libsdz_matches_python():
    """the C ABI's sdz_lpt_shard (used by sdz_*_batch_multi) is the same assignment"""
    import sdz
    rng = random.Random(9)
    for world in (1, 2, 3, 8):
        for n in (0, 1, 7, 500):
            sizes = [int(4096 * 2 ** rng.uniform(0, 12)) if k % 5 else 4096 for k in range(n)]
            owner = sdz.lpt_shard(sizes, world)
            shards = sdz_dist.lpt_shard(sizes, world)
            assert [sorted(i for i in range(n) if owner[i] == r) for r in range(world)] == shards


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


def _engine_worker(rank, world, port, q):
    """one rank: the real engine on this rank's LPT shard, the records all-gathered with the
    layout the C ABI's gather uses (sdz_dist.gather_records_comm, here over gloo); rank 0 also
    runs the whole batch in one call, the single-device reference for every record byte"""
    import torch.distributed as dist
    import sdz
    from test_gpu_multi import _mixed_batch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plain, comp = _mixed_batch(40, seed=21)
    shards = sdz_dist.lpt_shard([len(c) for c in comp], world)
    import ctypes

    def run(idx):
        n = len(idx)
        ins = (ctypes.c_char_p * n)(*[comp[i] for i in idx])
        in_len = (ctypes.c_size_t * n)(*[len(comp[i]) for i in idx])
        bufs = [ctypes.create_string_buffer(len(plain[i]) + 64) for i in idx]
        outs = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in bufs])
        caps = (ctypes.c_size_t * n)(*[len(plain[i]) + 64 for i in idx])
        recs = (sdz.InflateRecord * n)()
        assert sdz.lib().sdz_inflate_batch(ins, in_len, outs, caps, recs, n, sdz.FMT_AUTO, None, 0) == 0
        ok = all(bufs[k].raw[:recs[k].out_len] == plain[i] for k, i in enumerate(idx))
        return ok, bytes(recs)
    mine = shards[rank]
    ok, recs = run(mine)
    rsz = ctypes.sizeof(sdz.InflateRecord)
    allrec = sdz_dist.gather_records_comm(sdz_dist.TorchComm(), recs, rsz, shards)
    whole = None
    if rank == 0:
        wok, wrec = run(list(range(len(comp))))
        ok = ok and wok
        whole = [wrec[i * rsz:(i + 1) * rsz] for i in range(len(comp))]
    dist.destroy_process_group()
    q.put((rank, ok, allrec, whole))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_engine_shards_world2_gloo():
    import struct
    from test_gpu_multi import _mixed_batch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, ok, recs, whole = q.get(timeout=240)
        res[rank] = (ok, recs, whole)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    plain, _ = _mixed_batch(40, seed=21)
    whole = res[0][2]
    for rank in (0, 1):
        ok, recs, _ = res[rank]
        assert ok
        assert len(recs) == len(plain)
        for i, r in enumerate(recs):
            assert struct.unpack("<i", r[0:4])[0] == 0, i                   # SDZ_OK on every stream
            assert struct.unpack("<Q", r[8:16])[0] == len(plain[i]), i     # out_len, in stream order
            assert r == whole[i], i                                          # every byte of the record
