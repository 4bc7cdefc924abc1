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


def _pad(rec_bytes, rec_size, shards):
    """a rank's records padded to the largest shard: the fixed slot every rank contributes"""
    n_max = max(len(s) for s in shards)
    buf = bytearray(n_max * rec_size)
    buf[:len(rec_bytes)] = rec_bytes
    return bytes(buf)


def _reassemble(parts, rec_size, shards):
    """rank r's slot holds the records of shards[r] in order: back to stream order"""
    result = [None] * sum(len(s) for s in shards)
    for r, data in enumerate(parts):
        for k, i in enumerate(shards[r]):
            result[i] = data[k * rec_size:(k + 1) * rec_size]
    return result


class TorchComm:
    """sdz.Comm's allgather_bytes over torch.distributed (gloo on the CPU, or "nccl" with
    device="cuda"), so that tests run the gather's record layout without RCCL."""

    def __init__(self, device="cpu"):
        self.device = device

    def allgather_bytes(self, data):
        import torch
        import torch.distributed as dist
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(self.device)
        outs = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(outs, t)
        return [o.cpu().numpy().tobytes() for o in outs]


def gather_records_comm(comm, rec_bytes, rec_size, shards):
    """All-gather every rank's packed records (bytes, rec_size each, in its shard's order)
    over `comm` (sdz.Comm: RCCL inside libsdz; or TorchComm) and return the records of all
    streams in original order (list of bytes).  Ranks may hold different counts: each
    contributes a slot padded to the largest shard."""
    return _reassemble(comm.allgather_bytes(_pad(rec_bytes, rec_size, shards)), rec_size, shards)


def gather_records(rec_bytes, rec_size, shards, rank, device="cpu"):
    """gather_records_comm over torch.distributed (the process group already initialised)"""
    return gather_records_comm(TorchComm(device), rec_bytes, rec_size, shards)
