#!/usr/bin/env python3
"""Headline benchmark: batched inflate on MI355X (BASELINE.json configs[1], "C2").

A step = one pass of the hot path over one batch: 65,536 device-resident copies
of the reference fixture paradiselost.deflate (193,730 B -> 471,162 B each) are
inflated by the HIP kernel into their own output slots, checksums fused.  With
--gpus N (torchrun, one rank per GPU) every rank inflates its own 64 Ki streams
(weak scaling, no data-path collective); the per-stream result records are
all-gathered over RCCL inside libsdz after the timed region (gather_ms), and the
step barrier / max-over-ranks timing run over the same communicator.

Also reported: the kernel's HBM roofline fraction (HIP events on the launch
stream), the CPU baseline (oracle restatement on host cores; the reference's
own Node path cannot be run) and a deflate leg (configs[2]).
"""
import argparse
import ctypes
import glob
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

METRIC = ("uncompressed MB/s (inflate) + compressed MB/s (deflate) per node, 1/2/4/8 GPUs; "
          "% HBM roofline")
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def round_up(x, a):
    return (x + a - 1) // a * a


class DeviceBatch:
    """n device-resident streams replicated from one payload (no aliasing)."""

    def __init__(self, sdz, payload, n, out_cap, in_align=256):
        L = sdz.lib()
        self.sdz, self.n = sdz, n
        self.in_stride = round_up(len(payload), in_align)
        self.out_stride = round_up(out_cap, 256)
        self.d_in = sdz.DeviceBuffer(self.in_stride * n + 128)
        self.d_out = sdz.DeviceBuffer(self.out_stride * n + 64)
        self.d_in.upload(payload, 0)
        have = 1
        while have < n:                                   # doubling device-side replication
            k = min(have, n - have)
            rc = L.sdz_copy_device_to_device(self.d_in.ptr + have * self.in_stride, self.d_in.ptr,
                                             k * self.in_stride)
            assert rc == 0, L.sdz_last_error()
            have += k
        meta = []
        meta += [i * self.in_stride for i in range(n)]
        meta += [len(payload)] * n
        meta += [i * self.out_stride for i in range(n)]
        meta += [out_cap] * n
        arr = (ctypes.c_uint64 * len(meta))(*meta)
        self.d_meta = sdz.DeviceBuffer(8 * len(meta))
        self.d_meta.upload(bytes(arr))
        self.rec_size = ctypes.sizeof(sdz.InflateRecord)
        self.d_rec = sdz.DeviceBuffer(max(self.rec_size, ctypes.sizeof(sdz.DeflateRecord)) * n)

    def ptrs(self):
        m, n = self.d_meta.ptr, self.n
        return m, m + 8 * n, m + 16 * n, m + 24 * n

    def free(self):
        for b in (self.d_in, self.d_out, self.d_meta, self.d_rec):
            b.free()


def slice_offsets(n, span, seed=0x5D5A1B1E):
    """n slice offsets in [0, span) from a seeded xorshift64."""
    x, out = seed, []
    for _ in range(n):
        x ^= (x << 13) & 0xFFFFFFFFFFFFFFFF
        x ^= x >> 7
        x ^= (x << 17) & 0xFFFFFFFFFFFFFFFF
        out.append(x % span)
    return out


def fill_slices(sdz, b, text, offs, slice_len):
    """Stream j of batch b <- text[offs[j] : offs[j] + slice_len]: ONE k_gather launch
    (sdz_gather_device), not one copy dispatch per stream."""
    L = sdz.lib()
    n = len(offs)
    src = sdz.DeviceBuffer(len(text) + 64)
    src.upload(text)
    meta = [j * b.in_stride for j in range(n)] + list(offs) + [slice_len] * n
    d_meta = sdz.DeviceBuffer(8 * len(meta))
    d_meta.upload(bytes((ctypes.c_uint64 * len(meta))(*meta)))
    m = d_meta.ptr
    assert L.sdz_gather_device(b.d_in.ptr, m, src.ptr, m + 8 * n, m + 16 * n, n, None) == 0, L.sdz_last_error()
    assert L.sdz_sync(None) == 0
    src.free()
    d_meta.free()


def inflate_distinct(sdz, L, bd, drec, text, offs, slice_len, steps, barrier, allmax, world):
    """Inflate the deflate leg's n distinct compressed streams (device-resident) back into
    64 KiB slots: every stream has its own Huffman tables and LZ77 history."""
    n = bd.n
    in_len = [r.out_len for r in drec]
    meta = [j * bd.out_stride for j in range(n)] + in_len + \
           [j * round_up(slice_len, 256) for j in range(n)] + [slice_len] * n
    d_meta = sdz.DeviceBuffer(8 * len(meta))
    d_meta.upload(bytes((ctypes.c_uint64 * len(meta))(*meta)))
    d_out = sdz.DeviceBuffer(round_up(slice_len, 256) * n + 64)
    rec_size = ctypes.sizeof(sdz.InflateRecord)
    d_rec = sdz.DeviceBuffer(rec_size * n)
    m = d_meta.ptr

    def step(split):
        rc = L.sdz_inflate_batch_device(bd.d_out.ptr, m, m + 8 * n, d_out.ptr, m + 16 * n, m + 24 * n,
                                        d_rec.ptr, n, sdz.FMT_AUTO, None, 0, None)
        if rc:
            raise RuntimeError(L.sdz_last_error().decode())
        ms = L.sdz_last_kernel_ms()
        f3 = (ctypes.c_float * 3)()
        L.sdz_last_kernel_breakdown(f3)
        split.append(list(f3))
        return ms

    step([])
    L.sdz_sync(None)
    barrier()
    t0 = time.perf_counter()
    kms, split = [], []
    for _ in range(steps):
        kms.append(step(split))
    L.sdz_sync(None)
    barrier()
    wall = allmax(time.perf_counter() - t0) / steps
    recs = (sdz.InflateRecord * n).from_buffer_copy(d_rec.download(n * rec_size))
    ok = all(r.status == 0 and r.success and r.out_len == slice_len and r.checksum_verdict == 1 for r in recs)
    for j in sorted({0, n // 2, n - 1}):
        ok = ok and d_out.download(slice_len, j * round_up(slice_len, 256)) == text[offs[j]:offs[j] + slice_len]
    ok = allmax(0.0 if ok else 1.0) == 0.0
    # a sample of the compressed streams for the CPU baseline (the oracle inflating them)
    sample = [bd.d_out.download(in_len[j], j * bd.out_stride) for j in range(0, n, max(1, n // 256))]
    for x in (d_meta, d_out, d_rec):
        x.free()
    kernel_ms = sum(kms) / len(kms)
    bin_, bout = sum(in_len), n * slice_len
    achieved = (bin_ + bout) / (kernel_ms / 1000.0) / 1e9
    dtraffic = None                                       # rocprofv3 PMC pass of this leg (tools/run_c2.py --mode distinct)
    dps = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_distinct_pmc.json")))
    if dps and n == 65536 and slice_len == 65536:
        try:
            dtraffic = json.load(open(dps[-1])).get("hbm_bytes_per_launch")
        except Exception:
            dtraffic = None
    return {
        "value": round(world * bout / wall / 1e6, 2), "unit": "MB/s", "ms_per_step": round(1000 * wall, 3),
        "config": {"workload": "64 Ki distinct 64 KiB dynamic-Huffman zlib streams (the deflate leg's "
                               "outputs; north-star target)", "streams_per_gpu": n,
                   "bytes_in_per_gpu": bin_, "bytes_out_per_gpu": bout},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": dtraffic, "kernel_ms": round(kernel_ms, 3),
                     "kernels_ms": {"k_inflate_decode": round(sum(x[0] for x in split) / len(split), 3),
                                    "k_inflate_resolve": round(sum(x[1] for x in split) / len(split), 3),
                                    "k_inflate_finalize": round(sum(x[2] for x in split) / len(split), 3)}},
        "parity": bool(ok),
    }, sample


def inflate_step(sdz, b, split=None):
    in_off, in_len, out_off, out_cap = b.ptrs()
    rc = sdz.lib().sdz_inflate_batch_device(b.d_in.ptr, in_off, in_len, b.d_out.ptr, out_off, out_cap,
                                            b.d_rec.ptr, b.n, sdz.FMT_AUTO, None, 0, None)
    if rc:
        raise RuntimeError(sdz.lib().sdz_last_error().decode())
    ms = sdz.lib().sdz_last_kernel_ms()
    if split is not None:                                  # decode / resolve / finalize (HIP events)
        f3 = (ctypes.c_float * 3)()
        sdz.lib().sdz_last_kernel_breakdown(f3)
        split.append(list(f3))
    return ms


def deflate_step(sdz, b, level, fmt):
    in_off, in_len, out_off, out_cap = b.ptrs()
    rc = sdz.lib().sdz_deflate_batch_device(b.d_in.ptr, in_off, in_len, b.d_out.ptr, out_off, out_cap,
                                            b.d_rec.ptr, b.n, level, fmt, None, 0, 0, None, 0, None)
    if rc:
        raise RuntimeError(sdz.lib().sdz_last_error().decode())
    return sdz.lib().sdz_last_kernel_ms()


def deflate_fast_leg(sdz, L, text, offs, slice_len, nd, steps, barrier, allmax, world, rank):
    """The opt-in fast compressor (not bit-exact) on the C3 slices: valid
    zlib streams (checked with Python's zlib on a sample), throughput and ratio."""
    import zlib
    bf = DeviceBatch(sdz, text[:slice_len], nd, int(L.sdz_deflate_fast_bound(slice_len, 1, 0)))
    fill_slices(sdz, bf, text, offs, slice_len)

    def step():
        in_off, in_len, out_off, out_cap = bf.ptrs()
        if L.sdz_deflate_fast_batch_device(bf.d_in.ptr, in_off, in_len, bf.d_out.ptr, out_off, out_cap,
                                           bf.d_rec.ptr, nd, 1, None, 0, 0, None):
            raise RuntimeError(L.sdz_last_error().decode())
        return L.sdz_last_kernel_ms()
    step()
    L.sdz_sync(None)
    barrier()
    t0 = time.perf_counter()
    ks = [step() for _ in range(steps)]
    L.sdz_sync(None)
    barrier()
    wall = allmax(time.perf_counter() - t0) / steps
    rec = (sdz.DeflateRecord * nd).from_buffer_copy(bf.d_rec.download(nd * ctypes.sizeof(sdz.DeflateRecord)))
    total = sum(r.out_len for r in rec)
    ok = all(r.status == 0 for r in rec)
    if rank == 0:
        for j in sorted({0, 1, nd // 3, nd // 2, nd - 1}):
            ok = ok and zlib.decompress(bf.d_out.download(rec[j].out_len, j * bf.out_stride)) == \
                text[offs[j]:offs[j] + slice_len]
    bf.free()
    return {"value": round(world * total / wall / 1e6, 2), "unit": "compressed MB/s",
            "input_MBps": round(world * nd * slice_len / wall / 1e6, 2), "ratio": round(total / (nd * slice_len), 4),
            "kernel_ms": round(sum(ks) / len(ks), 3), "ms_per_step": round(1000 * wall, 3),
            "config": {"workload": "C3 slices, opt-in fast compressor (8 KiB tiles, greedy parse; NOT bit-exact)",
                       "streams_per_gpu": nd, "slice_bytes": slice_len},
            "valid": bool(ok), "bit_exact": False}


def mixed_leg(sdz, L, steps, scale, barrier, allmax, world, rank):
    """BASELINE configs[3] (C4) shape across the ranks: 262,144 streams of 4 KiB - 16 MiB
    (log-uniform, raw/zlib/gzip, compressible text) LPT-sharded over the node's 8 GPUs
    (sdz_dist.lpt_shard); rank r decodes every `scale`-th stream of shard r (weak scaling:
    at 8 ranks, 1/scale of the node's batch).  Streams are device copies of a pool of 36
    distinct payloads (12 size buckets x 3 formats), as in tools/run_configs.py."""
    import importlib.util
    import math
    import random
    import sdz_dist
    spec = importlib.util.spec_from_file_location("run_configs", os.path.join(ROOT, "tools", "run_configs.py"))
    rc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rc)
    lo, hi = math.log(4096), math.log(16 << 20)
    edges = [int(math.exp(lo + (hi - lo) * (k + 0.5) / 12)) for k in range(12)]
    rng = random.Random(0x5D5A1B1E)
    step = (hi - lo) / 12                                  # a size's bucket: the nearest edge (log scale)
    bucket = [min(11, int((rng.uniform(lo, hi) - lo) / step)) for _ in range(262144)]
    shards = sdz_dist.lpt_shard([edges[k] for k in bucket], 8)
    prng = random.Random(0x5D5A1B1F)
    pool, plain = [], []
    for k, sz in enumerate(edges):                         # pool index 3 k + format
        for fmt in range(3):
            data = rc.text(prng, sz)
            plain.append(data)
            pool.append(rc.compress(data, fmt))
    picks = [[3 * bucket[i] + i % 3 for i in shards[r % 8][::scale]] for r in range(world)]
    pick = picks[rank]
    caps = [len(plain[j]) + 64 for j in pick]
    slots = rc.Slots(pool, pick, caps)

    split = []

    def step():
        a, b, c, d = slots.ptrs()
        if L.sdz_inflate_batch_device(slots.d_in.ptr, a, b, slots.d_out.ptr, c, d, slots.d_rec.ptr, slots.n,
                                      sdz.FMT_AUTO, None, 0, None):
            raise RuntimeError(L.sdz_last_error().decode())
        ms = L.sdz_last_kernel_ms()
        f3 = (ctypes.c_float * 3)()                       # decode (incl. the split rounds) / resolve / finalize
        L.sdz_last_kernel_breakdown(f3)
        split.append(list(f3))
        return ms
    step()
    L.sdz_sync(None)
    barrier()
    split.clear()
    t0 = time.perf_counter()
    ks = [step() for _ in range(steps)]
    L.sdz_sync(None)
    barrier()
    wall = allmax(time.perf_counter() - t0) / steps
    recs = slots.records(sdz.InflateRecord)
    ok = all(recs[i].status == 0 and recs[i].success and recs[i].out_len == len(plain[j]) and
             (recs[i].checksum_verdict == 1 or j % 3 == 0) for i, j in enumerate(pick))
    seen = set()
    for i, j in enumerate(pick):                          # one stream per pool payload byte-compared
        if j not in seen:
            seen.add(j)
            ok = ok and slots.d_out.download(len(plain[j]), slots.out_off[i]) == plain[j]
    in_bytes = slots.in_bytes
    slots.free()
    ok = allmax(0.0 if ok else 1.0) == 0.0
    total_out = sum(len(plain[j]) for pk in picks for j in pk)
    total_in = sum(len(pool[j]) for pk in picks for j in pk)
    kms = sum(ks) / len(ks)
    kp = [sum(x[k] for x in split) / len(split) for k in range(3)]
    alg = in_bytes + sum(len(plain[j]) for j in pick)      # one rank's launch: compressed in + plain out
    mtraffic = None                                        # rocprofv3 PMC pass of this leg (tools/run_c2.py --mode mixed)
    mp = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_mixed_pmc.json")))
    if mp and world == 1 and scale == 8:
        try:
            mtraffic = json.load(open(mp[-1])).get("hbm_bytes_per_launch")
        except Exception:
            mtraffic = None
    achieved = alg / kms / 1e6
    return {"value": round(total_out / wall / 1e6, 2), "unit": "MB/s", "ms_per_step": round(1000 * wall, 3),
            "kernel_ms": round(kms, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": mtraffic,
                         "algorithmic_bytes_per_launch": alg,
                         "kernels_ms": {"k_inflate_decode": round(kp[0], 3), "k_inflate_resolve": round(kp[1], 3),
                                        "k_inflate_finalize": round(kp[2], 3),
                                        "other": round(max(0.0, kms - sum(kp)), 3)},
                         "launch": "one sdz_inflate_batch_device call: the lane / wave decoder and the block-split "
                                   "decoder rounds (k_split) in 'k_inflate_decode', resolve rounds, gzip crc32; "
                                   "'other': the rest of the launch (staging, copies)"},
            "config": {"workload": "C4 shape: 262,144 streams of 4 KiB-16 MiB (raw/zlib/gzip) LPT-sharded over 8 "
                                   "GPUs; each rank decodes every %dth stream of its shard" % scale,
                       "streams_per_gpu": len(pick), "bytes_out_all_ranks": total_out, "bytes_in_all_ranks": total_in,
                       "largest_stream_out": max(len(plain[j]) for j in pick)},
            "parity": bool(ok)}


def cpu_run(work_one, seconds, threads):
    """Run work_one(i) -> bytes counted, on `threads` host threads for `seconds` (the oracle
    releases the GIL inside its C calls).  Returns (units, bytes, elapsed s)."""
    counts, nbytes = [0] * threads, [0] * threads
    stop = time.perf_counter() + seconds

    def work(t):
        i = t
        while time.perf_counter() < stop:
            nbytes[t] += work_one(i)
            counts[t] += 1
            i += threads

    t0 = time.perf_counter()
    ths = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return sum(counts), sum(nbytes), time.perf_counter() - t0


def cpu_inflater(comps, out_cap):
    """work_one for cpu_run: the oracle (C restatement of the reference) inflating comps[i]"""
    import oracle as O
    L = O.lib()
    local = threading.local()

    def one(i):
        if not hasattr(local, "buf"):
            local.buf = ctypes.create_string_buffer(out_cap)
            local.res = O.InflateResult()
        c = comps[i % len(comps)]
        L.oracle_inflate(c, len(c), None, 0, local.buf, out_cap, ctypes.byref(local.res))
        assert local.res.success
        return local.res.total_out
    return one


def cpu_deflater(srcs, level):
    """work_one for cpu_run: the oracle's deflate(src, {level}) ("deflate" container);
    counts compressed bytes"""
    import oracle as O
    L = O.lib()
    local = threading.local()

    def one(i):
        src = srcs[i % len(srcs)]
        if not hasattr(local, "buf"):
            local.cap = len(src) + len(src) // 8 + 4096
            local.buf = ctypes.create_string_buffer(local.cap)
            local.olen = ctypes.c_size_t(0)
        parts = (ctypes.c_char_p * 1)(src)
        lens = (ctypes.c_size_t * 1)(len(src))
        err = L.oracle_deflater_run(parts, lens, 1, level, 1, None, 0, 0, None, 0, 0, local.buf, local.cap,
                                    ctypes.byref(local.olen))
        assert err == 0
        return local.olen.value
    return one


def cpu_threads():
    """Host threads for the CPU baseline: every core this process may run on, capped at the
    GPU box's CPU share for one GPU (OMP_NUM_THREADS, 16 there; the box's nproc counts the
    whole machine, whose other cores belong to the other GPUs' jobs)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(avail, int(share))) if share and share.isdigit() else max(1, avail), avail


def cgroup_cpu_limit():
    """The CPU quota of this process's cgroup (cgroup v2 cpu.max: "quota period", or "max"), as
    CPUs, or None when there is none: it caps what any number of threads can measure."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(work_one, seconds, unit_bytes_fn, sample):
    """The same work on the box's CPU share for one GPU (value), on one thread (per core), and on
    every core this process may run on (all_cores_measured_MBps: SURVEY §8(d)'s pool over all host
    cores, measured, beside the per-core x nproc extrapolation); MB/s of unit_bytes_fn"""
    threads, avail = cpu_threads()
    cnt, nb, dt = cpu_run(work_one, seconds, threads)
    c1, nb1, d1 = cpu_run(work_one, max(0.5, seconds / 2), 1)
    per_core = unit_bytes_fn(c1, nb1) / d1 / 1e6
    nproc = os.cpu_count() or 1
    if avail > threads:
        ca, nba, da = cpu_run(work_one, max(1.0, seconds / 2), avail)
        all_meas = unit_bytes_fn(ca, nba) / da / 1e6
    else:
        ca, da, all_meas = cnt, dt, unit_bytes_fn(cnt, nb) / dt / 1e6
    quota = cgroup_cpu_limit()
    return {"value": round(unit_bytes_fn(cnt, nb) / dt / 1e6, 2), "unit": "MB/s", "cores": threads, "kind": "port",
            "per_core_MBps": round(per_core, 2), "nproc": nproc, "affinity_cores": avail,
            "all_cores_measured_MBps": round(all_meas, 1), "all_cores_threads": max(avail, threads),
            "cgroup_cpu_quota": quota,
            "all_cores_linear_MBps": round(per_core * nproc, 1),
            "sample": "%s: %d units on %d threads in %.1f s; per core: %d in %.1f s on 1 thread; all cores: %d in "
                      "%.1f s on %d threads (every CPU in this process's affinity mask; cgroup quota %s CPUs); "
                      "threads = the box's CPU share for one GPU (OMP_NUM_THREADS) of nproc %d; "
                      "all_cores_linear_MBps = per-core x nproc, the machine-wide ceiling"
                      % (sample, cnt, threads, dt, c1, d1, ca, da, max(avail, threads), quota, nproc)}


def node_facade():
    """The reference's perf case (test/perf.html:54-87: 20 samples of deflate(paradiselost.txt,
    {level: 4}) and inflate(paradiselost.gz), extremes dropped) and C1 inflate(simple.deflate),
    through the drop-in ES module under Node (tests/node/perf.mjs); ms."""
    import shutil
    import subprocess
    node = shutil.which("node")
    addon = os.path.join(ROOT, "sd-zlib_amd", "js", "sdz_napi.node")
    if node is None or not os.path.exists(addon):
        return {"skipped": "node or the N-API addon is not available"}
    r = subprocess.run([node, os.path.join(ROOT, "tests", "node", "perf.mjs")], capture_output=True, text=True,
                       timeout=300)
    if r.returncode != 0:
        return {"error": (r.stderr or r.stdout)[-400:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def small_batch_leg(sdz, L, comp, text, n, steps):
    """A small batch (n copies of C2's stream): the wave decoder (a wave per stream, picked by
    inflate_wave_policy for batches of at most 65,536 streams whose longest is 16 KiB - 4 MiB of
    input and whose total is at most 24,576 times the longest) against the lane path
    (SDZ_WDEC=0: a lane per stream, its time the longest stream's serial decode, or the
    block-parallel split of the streams where its cost model picks it); kernel ms."""
    b = DeviceBatch(sdz, comp, n, len(text) + 64)
    res = {"streams": n, "bytes_out": n * len(text)}
    try:
        for name, env in (("wave", None), ("lane", "0")):
            old = os.environ.pop("SDZ_WDEC", None)
            if env is not None:
                os.environ["SDZ_WDEC"] = env
            try:
                inflate_step(sdz, b)
                split = []
                ms = [inflate_step(sdz, b, split) for _ in range(steps)]
            finally:
                os.environ.pop("SDZ_WDEC", None)
                if old is not None:
                    os.environ["SDZ_WDEC"] = old
            recs = (sdz.InflateRecord * n).from_buffer_copy(b.d_rec.download(n * b.rec_size))
            ok = all(r.success and r.out_len == len(text) for r in recs) and \
                all(b.d_out.download(len(text), j * b.out_stride) == text for j in (0, n - 1))
            kms = sum(ms) / len(ms)
            res[name] = {"kernel_ms": round(kms, 3), "GBps_out": round(n * len(text) / kms / 1e6, 1),
                         "decode_ms": round(sum(x[0] for x in split) / len(split), 3),
                         "resolve_ms": round(sum(x[1] for x in split) / len(split), 3), "parity": bool(ok)}
    finally:
        b.free()
    return res


def facade_latency(sdz, reps=40):
    """BASELINE configs[0] (C1) through the drop-in's host path: inflate(simple.deflate) and
    deflate(simple.txt) one call at a time (staging pools, no per-call allocation); median
    microseconds per call.  Also deflate(paradiselost.txt) at L1/L6/L9 (test/perf.html's
    case), checked against the reference fixture (L6) and the published size table."""
    golden = os.path.join(ROOT, "tests", "golden")
    simple_c = open(os.path.join(golden, "simple.deflate"), "rb").read()
    simple_t = open(os.path.join(golden, "simple.txt"), "rb").read()
    text = open(os.path.join(golden, "paradiselost.txt"), "rb").read()
    comp = open(os.path.join(golden, "paradiselost.deflate"), "rb").read()

    def med(f, k=reps):
        f()
        ts = []
        for _ in range(k):
            t0 = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2]
    ok = sdz.inflate(simple_c) == simple_t and sdz.deflate(simple_t, {"level": 6}) == simple_c
    res = {"inflate_simple_us": round(1e6 * med(lambda: sdz.inflate(simple_c)), 1),
           "deflate_simple_us": round(1e6 * med(lambda: sdz.deflate(simple_t, {"level": 6})), 1),
           "inflate_paradiselost_ms": round(1e3 * med(lambda: sdz.inflate(comp)), 3)}
    sizes = {1: 226188, 6: 193730, 9: 193162}           # test/perf.html:63-69
    for lv in (1, 6, 9):
        out = sdz.deflate(text, {"level": lv})
        ok = ok and len(out) == sizes[lv] and (lv != 6 or out == comp)
        res["deflate_paradiselost_L%d_ms" % lv] = round(1e3 * med(lambda: sdz.deflate(text, {"level": lv}), 5), 3)
    res["parity"] = bool(ok)
    res["note"] = ("drop-in facade (Python mirror of sd-inflate.ts / sd-deflate.ts) over the host-buffer C ABI; "
                   "reference browser times for deflate(paradiselost.txt): L1 15-22 ms, L6 39-48 ms, L9 49-57 ms "
                   "(test/perf.html:63-69)")
    return res


class Ranks:
    """One process per GPU (torchrun env).  The collectives run over RCCL inside libsdz
    (sdz_comm_*): the step barrier, max-over-ranks timing and the record all-gather.  The
    only other channel is gloo on the CPU, used once to hand rank 0's RCCL id to the others."""

    def __init__(self, sdz):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.comm = None
        if self.world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            box = [sdz.Comm.unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            self.comm = sdz.Comm(box[0], self.world, self.rank)
            self.dist = dist

    def barrier(self):
        if self.comm:
            self.comm.max(0.0)

    def allmax(self, x):
        return self.comm.max(x) if self.comm else x

    def close(self):
        if self.comm:
            self.comm.close()
            self.dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--streams", type=int, default=65536, help="streams per GPU (C2: 65536)")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--deflate-streams", type=int, default=65536,
                    help="streams for the deflate leg (64 KiB slices, L6); 0 disables")
    ap.add_argument("--deflate-steps", type=int, default=3)
    ap.add_argument("--fast-steps", type=int, default=2,
                    help="steps of the opt-in fast (not bit-exact) compressor leg on the C3 slices (0: skip)")
    ap.add_argument("--distinct-steps", type=int, default=3,
                    help="steps of the distinct-stream inflate leg (the deflate leg's outputs); 0 disables")
    ap.add_argument("--mixed-steps", type=int, default=2,
                    help="steps of the C4-shaped mixed-size leg (LPT shards of 262,144 streams; 0: skip)")
    ap.add_argument("--mixed-scale", type=int, default=8,
                    help="the mixed leg decodes every Nth stream of the rank's LPT shard (1: the full shard)")
    ap.add_argument("--copy-gib", type=float, default=4.0, help="device copy peak probe size; 0 disables")
    ap.add_argument("--host-streams", type=int, default=0,
                    help="streams for the host-buffer (PCIe-inclusive) inflate probe, e.g. 2048; off by "
                         "default so that the rocprofv3 stats of the default command hold C2 launches only")
    ap.add_argument("--latency", type=int, default=1, help="C1-style single-call latency of the facade (0: skip)")
    ap.add_argument("--small-streams", type=int, default=1024,
                    help="small-batch leg: that many copies of C2's stream, wave vs lane decoder (0: skip)")
    ap.add_argument("--node", type=int, default=1,
                    help="time the reference's own perf case (test/perf.html) through the Node facade (0: skip)")
    args = ap.parse_args()

    # --gpus N (N > 1) outside torchrun: one rank per GPU under torch.distributed.run, started
    # as a child process before anything touches a GPU; this process exits with its code
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import socket
        import subprocess
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        log("bench.py: --gpus %d -> %s" % (args.gpus, " ".join(cmd)))
        raise SystemExit(subprocess.call(cmd))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        log("bench.py: WORLD_SIZE=%s differs from --gpus %d; n_gpus reports the ranks that ran"
            % (os.environ.get("WORLD_SIZE"), args.gpus))

    import sdz
    L = sdz.lib()
    if sdz.device_count() < 1:
        raise SystemExit("bench.py: no GPU visible")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert L.sdz_set_device(local) == 0
    R = Ranks(sdz)
    rank, world = R.rank, R.world
    barrier, allmax = R.barrier, R.allmax

    golden = os.path.join(ROOT, "tests", "golden")
    comp = open(os.path.join(golden, "paradiselost.deflate"), "rb").read()
    text = open(os.path.join(golden, "paradiselost.txt"), "rb").read()
    n = args.streams
    b = DeviceBatch(sdz, comp, n, len(text))
    L.sdz_set_timing(1)
    for _ in range(args.warmup):
        inflate_step(sdz, b)
    L.sdz_sync(None)
    barrier()
    L.sdz_sync(None)
    kms, split = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        kms.append(inflate_step(sdz, b, split))
    L.sdz_sync(None)
    barrier()
    t1 = time.perf_counter()
    wall = allmax(t1 - t0)
    ms_per_step = 1000.0 * wall / args.steps
    kernel_ms = sum(kms) / len(kms)

    # ---- parity of the timed outputs (records + sampled payloads)
    recs = (sdz.InflateRecord * n).from_buffer_copy(b.d_rec.download(n * b.rec_size))
    ok = all(r.status == 0 and r.success and r.out_len == len(text) and r.checksum_verdict == 1 for r in recs)
    for i in sorted({0, n // 3, n - 1}):
        ok = ok and b.d_out.download(len(text), i * b.out_stride) == text
    # ---- RCCL all-gather of the per-stream result records (libsdz; outside the timed region)
    gather_ms = None
    if world > 1:
        import sdz_dist
        shards = [list(range(r * n, (r + 1) * n)) for r in range(world)]   # weak scaling: n per rank
        g0 = time.perf_counter()
        allrec = sdz_dist.gather_records_comm(R.comm, bytes(recs), b.rec_size, shards)
        gather_ms = 1000.0 * (time.perf_counter() - g0)
        ok = ok and len(allrec) == world * n and all(
            sdz.InflateRecord.from_buffer_copy(r).status == 0 and sdz.InflateRecord.from_buffer_copy(r).success
            for r in allrec)
    okall = allmax(0.0 if ok else 1.0) == 0.0
    bytes_in, bytes_out = len(comp) * n, len(text) * n
    b.free()

    # ---- measured device copy peak (report against it in the same run):
    # k_gather (sdz_gather_device) moving copy_gib of 1 MiB spans, timed with HIP events
    copy_gbs = None
    if args.copy_gib > 0:
        nb = int(args.copy_gib * (1 << 30)) & ~((1 << 20) - 1)
        ns = nb >> 20
        src, dst = sdz.DeviceBuffer(nb), sdz.DeviceBuffer(nb)
        offs = [i << 20 for i in range(ns)]
        meta = offs + offs + [1 << 20] * ns
        d_meta = sdz.DeviceBuffer(8 * len(meta))
        d_meta.upload(bytes((ctypes.c_uint64 * len(meta))(*meta)))
        m = d_meta.ptr
        best = None
        for _ in range(4):
            assert L.sdz_gather_device(dst.ptr, m, src.ptr, m + 8 * ns, m + 16 * ns, ns, None) == 0
            ms = L.sdz_last_kernel_ms()
            best = ms if best is None else min(best, ms)
        copy_gbs = 2.0 * nb / (best / 1000.0) / 1e9              # read + write bytes
        for x in (src, dst, d_meta):
            x.free()

    # ---- host-buffer path (PCIe-inclusive, never `value`): sdz.inflate_batch on host bytes
    host = None
    if rank == 0 and args.host_streams > 0:
        hn = args.host_streams
        ins = (ctypes.c_char_p * hn)(*([comp] * hn))
        in_len = (ctypes.c_size_t * hn)(*([len(comp)] * hn))
        hbufs = [ctypes.create_string_buffer(len(text)) for _ in range(hn)]
        outs = (ctypes.c_void_p * hn)(*[ctypes.addressof(x) for x in hbufs])
        caps = (ctypes.c_size_t * hn)(*([len(text)] * hn))
        hrec = (sdz.InflateRecord * hn)()
        hdt = None
        for _ in range(2):                                  # the first call sizes the pools
            h0 = time.perf_counter()
            hrc = L.sdz_inflate_batch(ins, in_len, outs, caps, hrec, hn, sdz.FMT_AUTO, None, 0)
            hdt = time.perf_counter() - h0
        hok = hrc == 0 and all(r.success and r.out_len == len(text) for r in hrec) and \
            all(hbufs[i].raw == text for i in (0, hn - 1))
        host = {"streams": hn, "MBps_out": round(hn * len(text) / hdt / 1e6, 2),
                "seconds": round(hdt, 3), "parity": bool(hok),
                "note": "sdz_inflate_batch on host buffers: H2D + kernels + D2H, PCIe-inclusive"}
        del hbufs

    # ---- deflate leg (configs[2]: 64 KiB text slices, level 6, "deflate" container); every
    # stream is a distinct slice (xorshift64 offsets), and the compressed outputs then feed
    # the distinct-stream inflate leg (the north star's 64 Ki x 64 KiB dynamic-Huffman target)
    deflate = None
    distinct = None
    fast = None
    if args.deflate_streams > 0:
        nd = args.deflate_streams
        slice_len = 65536
        offs = slice_offsets(nd, len(text) - slice_len)
        bd = DeviceBatch(sdz, text[:slice_len], nd, int(L.sdz_deflate_bound(slice_len, 1, 0)))
        fill_slices(sdz, bd, text, offs, slice_len)
        deflate_step(sdz, bd, 6, 1)
        L.sdz_sync(None)
        barrier()
        d0 = time.perf_counter()
        dk = [deflate_step(sdz, bd, 6, 1) for _ in range(args.deflate_steps)]
        L.sdz_sync(None)
        barrier()
        dwall = allmax(time.perf_counter() - d0) / args.deflate_steps
        drec = (sdz.DeflateRecord * nd).from_buffer_copy(bd.d_rec.download(nd * ctypes.sizeof(sdz.DeflateRecord)))
        comp_total = sum(r.out_len for r in drec)
        dok = all(r.status == 0 for r in drec)
        if rank == 0:
            import oracle as O
            for j in sorted({0, 1, nd // 2, nd - 1}):
                got = bd.d_out.download(drec[j].out_len, j * bd.out_stride)
                dok = dok and got == O.deflate(text[offs[j]:offs[j] + slice_len], level=6)
        dkms = sum(dk) / len(dk)
        dalg = nd * slice_len + comp_total                  # uncompressed in + compressed out
        dachieved = dalg / (dkms / 1000.0) / 1e9
        dtraffic = None
        dpmcs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_deflate_pmc.json")))
        if dpmcs and nd == 65536:
            try:
                dtraffic = json.load(open(dpmcs[-1])).get("hbm_bytes_per_launch")
            except Exception:
                dtraffic = None
        deflate = {
            "value": round(world * comp_total / dwall / 1e6, 2), "unit": "compressed MB/s",
            "input_MBps": round(world * nd * slice_len / dwall / 1e6, 2),
            "kernel_ms": round(dkms, 3), "ms_per_step": round(1000 * dwall, 3),
            "config": {"workload": "C3 deflate level=6 format=deflate", "streams_per_gpu": nd,
                       "slice_bytes": slice_len,
                       "data": "%d distinct paradiselost.txt slices at xorshift64 offsets (enwik8 absent offline)" % nd},
            "roofline": {"bound": "hbm", "achieved": round(dachieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(dachieved / HBM_PEAK_GBS, 5), "traffic": dtraffic,
                         "algorithmic_bytes_per_launch": dalg,
                         "launch": "one sdz_deflate_batch_device call: k_dfl_chain/match/tail/parse/trees/encode "
                                   "(+ checksum), HIP events on the launch stream"},
            "parity": bool(dok),
        }
        if rank == 0 and world == 1 and args.cpu_seconds > 0:
            srcs = [text[offs[j]:offs[j] + slice_len] for j in range(0, nd, max(1, nd // 64))]
            deflate["cpu_baseline"] = cpu_baseline(
                cpu_deflater(srcs, 6), args.cpu_seconds, lambda c, nb: nb,
                "oracle C restatement deflate(L6, \"deflate\") of %d of the leg's 64 KiB slices, compressed MB/s"
                % len(srcs))
            deflate["cpu_baseline"]["input_MBps"] = None
        if args.distinct_steps > 0:
            distinct, dsample = inflate_distinct(sdz, L, bd, drec, text, offs, slice_len, args.distinct_steps,
                                                 barrier, allmax, world)
            if rank == 0 and world == 1 and args.cpu_seconds > 0:
                distinct["cpu_baseline"] = cpu_baseline(
                    cpu_inflater(dsample, slice_len + 64), args.cpu_seconds, lambda c, nb: nb,
                    "oracle C restatement inflating %d of the leg's distinct 64 KiB streams, uncompressed MB/s"
                    % len(dsample))
        bd.free()
        if args.fast_steps > 0 and hasattr(L, "sdz_deflate_fast_batch_device"):
            fast = deflate_fast_leg(sdz, L, text, offs, slice_len, nd, args.fast_steps, barrier, allmax, world, rank)

    mixed = None
    if args.mixed_steps > 0:
        mixed = mixed_leg(sdz, L, args.mixed_steps, args.mixed_scale, barrier, allmax, world, rank)

    small = None
    if rank == 0 and args.small_streams > 0:
        small = small_batch_leg(sdz, L, comp, text, args.small_streams, 3)
    latency = None
    if rank == 0 and args.latency > 0:
        # as a user calls it: without the kernel-time events the legs above read (each event is
        # a marker in the stream that the call's final wait also waits for)
        L.sdz_set_timing(0)
        latency = facade_latency(sdz)
        L.sdz_set_timing(1)
    nodef = None
    if rank == 0 and args.node > 0:
        nodef = node_facade()

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(cpu_inflater([comp], len(text) + 64), args.cpu_seconds, lambda c, nb: nb,
                           "paradiselost.deflate inflated by the oracle C restatement, uncompressed MB/s")

    traffic = None
    # the latest round's PMC traffic summary (tools/pmc_traffic.py over tools/profile_inflate.sh passes: profiles/rNN_inflate_pmc.json)
    pmcs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_inflate_pmc.json")))
    pmc = pmcs[-1] if pmcs else ""
    if pmc and os.path.exists(pmc) and n == 65536:
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    achieved = (bytes_in + bytes_out) / (kernel_ms / 1000.0) / 1e9
    kparts = [sum(x[k] for x in split) / len(split) for k in range(3)]
    line = {
        "metric": METRIC,
        "value": round(world * bytes_out / (wall / args.steps) / 1e6, 2),
        "unit": "MB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: 65536 device copies/GPU of reference fixture paradiselost.deflate",
        "config": {"workload": "C2 batched inflate: paradiselost.deflate x %d per GPU (zlib, dynamic Huffman)" % n,
                   "streams_per_gpu": n, "bytes_in_per_gpu": bytes_in, "bytes_out_per_gpu": bytes_out,
                   "parallelism": "dp%d (independent streams, no data-path collective; records all-gathered "
                                  "over RCCL inside libsdz)" % world},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "kernel_ms": round(kernel_ms, 3),
                     "kernels_ms": {"k_inflate_decode": round(kparts[0], 3),
                                    "k_inflate_resolve": round(kparts[1], 3),
                                    "k_inflate_finalize": round(kparts[2], 3)},
                     "launch": "one sdz_inflate_batch_device call = decode + resolve + finalize kernels",
                     "algorithmic_bytes_per_launch": bytes_in + bytes_out,
                     "measured_copy_GBps": None if copy_gbs is None else round(copy_gbs, 1),
                     "frac_of_copy": None if copy_gbs is None else round(achieved / copy_gbs, 5)},
        "host_path": host,
        "cpu_baseline": cpu,
        "parity": bool(okall),
        "gather_ms": None if gather_ms is None else round(gather_ms, 3),
        "deflate": deflate,
        "deflate_fast": fast,
        "inflate_distinct": distinct,
        "mixed": mixed,
        "facade_latency": latency,
        "inflate_small_batch": small,
        "node_facade": nodef,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    R.close()


if __name__ == "__main__":
    main()
