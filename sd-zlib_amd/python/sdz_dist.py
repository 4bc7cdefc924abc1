"""Multi-GPU host logic: one process per GPU, independent streams.

Streams never exchange data while they are decoded, so a batch is split across
ranks by size (LPT: largest first, onto the rank with the fewest bytes so far) and
each rank runs the single-GPU C ABI on its shard.  The only collective is the
all-gather of the fixed-size per-stream records at the end (RCCL on GPUs via the
"nccl" backend; gloo in the CPU tests), after which every rank can reassemble the
records in the original stream order.  With the engine's own communicator (sdz.Comm: RCCL
inside libsdz, one rank per process) the gather never touches torch.distributed.
"""
import heapq


def lpt_shard(sizes, world):
    """Assign stream indices to ranks: largest first onto the least-loaded rank.
    Returns one ascending index list per rank (deterministic for equal sizes)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    heap = [(0, r) for r in range(world)]
    shards = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda k: (-sizes[k], k)):
        load, r = heapq.heappop(heap)
        shards[r].append(i)
        heapq.heappush(heap, (load + sizes[i], r))
    return [sorted(s) for s in shards]


def gather_records(rec_bytes, rec_size, shards, rank, device="cpu"):
    """All-gather every rank's packed records (bytes, rec_size each, in its shard's
    order) and return the records of all streams in original order (list of bytes).
    Ranks may hold different counts: records are padded to the largest shard."""
    import torch
    import torch.distributed as dist
    world = len(shards)
    n_max = max(len(s) for s in shards)
    buf = bytearray(n_max * rec_size)
    buf[:len(rec_bytes)] = rec_bytes
    t = torch.frombuffer(buf, dtype=torch.uint8).to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    total = sum(len(s) for s in shards)
    result = [None] * total
    for r in range(world):
        data = outs[r].cpu().numpy().tobytes()
        for k, i in enumerate(shards[r]):
            result[i] = data[k * rec_size:(k + 1) * rec_size]
    return result


def gather_records_comm(comm, rec_bytes, rec_size, shards):
    """gather_records over libsdz's RCCL communicator (sdz.Comm.allgather_bytes)."""
    n_max = max(len(s) for s in shards)
    buf = bytearray(n_max * rec_size)
    buf[:len(rec_bytes)] = rec_bytes
    parts = comm.allgather_bytes(bytes(buf))
    result = [None] * sum(len(s) for s in shards)
    for r, data in enumerate(parts):
        for k, i in enumerate(shards[r]):
            result[i] = data[k * rec_size:(k + 1) * rec_size]
    return result
