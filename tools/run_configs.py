#!/usr/bin/env python3
"""BASELINE.json configs[3] (C4) and configs[4] (C5) at one GPU's share of the node.

Not the headline bench (bench.py measures C2 and C3); this measures the two other
batched configurations so that every BASELINE config has a number:

  C4  mixed batched inflate: 262,144 streams over 8 GPUs -> 32,768 per GPU.  Sizes are
      log-uniform in [4 KiB, 16 MiB] (seeded); formats cycle raw / zlib / gzip; content is
      compressible synthetic text.  A pool of distinct payloads per (size bucket, format),
      compressed once on the host by Python's zlib (an independent encoder), is replicated
      on the device.  Every stream is checked against its original bytes (device compare of
      lengths + sampled downloads) and every record must say success with checksum "match"
      (raw: "unchecked").
  C5  gzip round trip: 1 Mi x 32 KiB over 8 GPUs -> 131,072 per GPU.  64 distinct synthetic
      text payloads, deflated on the GPU at level 9, format gzip, mtime 0; the GPU output is
      inflated on the GPU; every record's checksum must be "match" and a sample of the
      deflate outputs must equal the oracle's bytes (bit-exact vs the reference restatement).

--scale divides the stream counts (default 1 = the full per-GPU share).  Prints one JSON
line per config.
  python3 tools/run_configs.py --config c4 --scale 16
"""
import argparse
import ctypes
import json
import math
import os
import random
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import sdz  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def text(rng, n):
    """Compressible synthetic text: words of the reference fixture, reshuffled."""
    words = open(os.path.join(GOLDEN, "paradiselost.txt"), "rb").read().split()
    out = bytearray()
    while len(out) < n:
        k = rng.randrange(len(words) - 64)
        out += b" ".join(words[k:k + rng.randint(4, 64)]) + (b".\n" if rng.random() < 0.2 else b" ")
    return bytes(out[:n])


def compress(data, fmt):
    if fmt == 0:                                          # raw DEFLATE
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        return c.compress(data) + c.flush()
    if fmt == 1:
        return zlib.compress(data, 6)                     # zlib container
    c = zlib.compressobj(6, zlib.DEFLATED, 31)            # gzip container
    return c.compress(data) + c.flush()


class Slots:
    """n device-resident streams laid out from a host pool (device copies of pool items)."""

    def __init__(self, pool, pick, out_caps, align=256):
        L = sdz.lib()
        self.n = len(pick)
        up = lambda x: (x + align - 1) // align * align  # noqa: E731
        self.pool_off, off = [], 0
        for p in pool:
            self.pool_off.append(off)
            off += up(len(p))
        self.d_pool = sdz.DeviceBuffer(off + 128)
        for p, o in zip(pool, self.pool_off):
            self.d_pool.upload(p, o)
        self.in_off, self.in_len, o = [], [], 0
        for j in pick:
            self.in_off.append(o)
            self.in_len.append(len(pool[j]))
            o += up(len(pool[j]))
        self.d_in = sdz.DeviceBuffer(o + 128)
        # every stream's copy of its pool payload in one k_gather launch (sdz_gather_device)
        gm = self.in_off + [self.pool_off[j] for j in pick] + self.in_len
        d_gm = sdz.DeviceBuffer(8 * max(1, len(gm)))
        d_gm.upload(bytes((ctypes.c_uint64 * len(gm))(*gm)))
        k = self.n
        rc = L.sdz_gather_device(self.d_in.ptr, d_gm.ptr, self.d_pool.ptr, d_gm.ptr + 8 * k, d_gm.ptr + 16 * k, k, None)
        assert rc == 0 and L.sdz_sync(None) == 0, L.sdz_last_error()
        d_gm.free()
        self.out_off, self.out_cap, o = [], [], 0
        for c in out_caps:
            self.out_off.append(o)
            self.out_cap.append(c)
            o += up(c)
        self.d_out = sdz.DeviceBuffer(o + 128)
        meta = self.in_off + self.in_len + self.out_off + self.out_cap
        self.d_meta = sdz.DeviceBuffer(8 * len(meta))
        self.d_meta.upload(bytes((ctypes.c_uint64 * len(meta))(*meta)))
        self.d_rec = sdz.DeviceBuffer(64 * self.n)
        self.in_bytes = sum(self.in_len)

    def ptrs(self):
        m, n = self.d_meta.ptr, self.n
        return m, m + 8 * n, m + 16 * n, m + 24 * n

    def records(self, cls):
        raw = self.d_rec.download(ctypes.sizeof(cls) * self.n)
        return (cls * self.n).from_buffer_copy(raw)

    def free(self):
        for b in (self.d_pool, self.d_in, self.d_out, self.d_meta, self.d_rec):
            b.free()


def inflate(slots, fmt):
    L = sdz.lib()
    a, b, c, d = slots.ptrs()
    t0 = time.perf_counter()
    rc = L.sdz_inflate_batch_device(slots.d_in.ptr, a, b, slots.d_out.ptr, c, d, slots.d_rec.ptr, slots.n,
                                    fmt, None, 0, None)
    L.sdz_sync(None)
    wall = (time.perf_counter() - t0) * 1e3
    assert rc == 0, L.sdz_last_error()
    f3 = (ctypes.c_float * 3)()
    L.sdz_last_kernel_breakdown(f3)
    log("inflate: decode %.2f ms (split pre-pass included), resolve %.2f ms, finalize %.2f ms" % tuple(f3))
    return L.sdz_last_kernel_ms(), wall


def run_c4(scale, seed=0x5D5A1B1E):
    rng = random.Random(seed)
    n = 32768 // scale
    lo, hi = math.log(4096), math.log(16 << 20)
    sizes = [int(math.exp(rng.uniform(lo, hi))) for _ in range(n)]
    # pool: 12 size buckets x 3 formats, one distinct payload each (a stream uses its bucket's
    # payload cut to its own size bucket edge: every stream's size is the bucket size)
    edges = [int(math.exp(lo + (hi - lo) * (k + 0.5) / 12)) for k in range(12)]
    pool, plain, key = [], [], {}
    t0 = time.perf_counter()
    for k, sz in enumerate(edges):
        for fmt in range(3):
            data = text(rng, sz)
            key[(k, fmt)] = len(pool)
            plain.append(data)
            pool.append(compress(data, fmt))
    log("c4: pool of %d payloads compressed in %.1f s" % (len(pool), time.perf_counter() - t0))
    pick = []
    for i, sz in enumerate(sizes):
        k = min(range(12), key=lambda j: abs(math.log(edges[j]) - math.log(sz)))
        pick.append(key[(k, i % 3)])
    caps = [len(plain[j]) + 64 for j in pick]
    slots = Slots(pool, pick, caps)
    out_bytes = sum(len(plain[j]) for j in pick)
    inflate(slots, sdz.FMT_AUTO)                          # warm-up
    kms, wall = inflate(slots, sdz.FMT_AUTO)
    recs = slots.records(sdz.InflateRecord)
    ok = all(recs[i].status == 0 and recs[i].success and recs[i].out_len == len(plain[pick[i]])
             and (recs[i].checksum_verdict == 1 or i % 3 == 0) for i in range(n))
    # sampled byte compare: one stream per pool item
    seen = set()
    for i, j in enumerate(pick):
        if j in seen:
            continue
        seen.add(j)
        got = slots.d_out.download(len(plain[j]), slots.out_off[i])
        ok = ok and got == plain[j]
    slots.free()
    biggest = max(len(plain[j]) for j in pick)
    return {"config": "C4 mixed batched inflate (per-GPU share of 262,144 streams / 8 GPUs)",
            "streams": n, "scale": "1/%d" % scale, "bytes_in": slots.in_bytes, "bytes_out": out_bytes,
            "largest_stream_out": biggest, "kernel_ms": round(kms, 3), "wall_ms": round(wall, 3),
            "uncompressed_MBps": round(out_bytes / kms / 1e3, 2),
            "roofline_GBps": round((slots.in_bytes + out_bytes) / kms / 1e6, 2),
            "parity": bool(ok), "checked": "every record (status, success, length, checksum match); "
            "one stream per pool item byte-compared with the original"}


def run_c5(scale, seed=0x5D5A1B1E):
    import oracle as O
    L = sdz.lib()
    rng = random.Random(seed)
    n = 131072 // scale
    pool = [text(rng, 32768) for _ in range(64)]
    pick = [i % 64 for i in range(n)]
    bound = int(L.sdz_deflate_bound(32768, 2, 0))
    slots = Slots(pool, pick, [bound] * n)
    a, b, c, d = slots.ptrs()
    rc = L.sdz_deflate_batch_device(slots.d_in.ptr, a, b, slots.d_out.ptr, c, d, slots.d_rec.ptr, n, 9, 2,
                                    None, 0, 0, None, 0, None)
    assert rc == 0, L.sdz_last_error()
    L.sdz_sync(None)                                      # the warm-up is asynchronous
    t0 = time.perf_counter()
    rc = L.sdz_deflate_batch_device(slots.d_in.ptr, a, b, slots.d_out.ptr, c, d, slots.d_rec.ptr, n, 9, 2,
                                    None, 0, 0, None, 0, None)
    L.sdz_sync(None)
    dwall = (time.perf_counter() - t0) * 1e3
    assert rc == 0, L.sdz_last_error()
    dms = L.sdz_last_kernel_ms()
    drecs = slots.records(sdz.DeflateRecord)
    ok = all(drecs[i].status == 0 for i in range(n))
    comp = []
    for i in range(64):                                   # bit-exact vs the oracle, one per payload
        got = slots.d_out.download(drecs[i].out_len, slots.out_off[i])
        comp.append(got)
        ok = ok and got == O.deflate(pool[i], level=9, format="gzip", mtime=0)
    cbytes = sum(drecs[i].out_len for i in range(n))
    # inflate the GPU's own output on the GPU
    islots = Slots(comp, pick, [32768 + 64] * n)
    inflate(islots, sdz.FMT_AUTO)
    ims, iwall = inflate(islots, sdz.FMT_AUTO)
    irecs = islots.records(sdz.InflateRecord)
    ok = ok and all(irecs[i].success and irecs[i].checksum_verdict == 1 and irecs[i].out_len == 32768
                    for i in range(n))
    for i in range(64):
        ok = ok and islots.d_out.download(32768, islots.out_off[i]) == pool[i]
    slots.free()
    islots.free()
    return {"config": "C5 gzip round trip level 9 (per-GPU share of 1 Mi x 32 KiB / 8 GPUs)",
            "streams": n, "scale": "1/%d" % scale, "bytes_in": 32768 * n, "bytes_compressed": cbytes,
            "deflate_kernel_ms": round(dms, 3), "deflate_wall_ms": round(dwall, 3),
            "deflate_input_MBps": round(32768 * n / dms / 1e3, 2),
            "deflate_compressed_MBps": round(cbytes / dms / 1e3, 2),
            "inflate_kernel_ms": round(ims, 3), "inflate_uncompressed_MBps": round(32768 * n / ims / 1e3, 2),
            "parity": bool(ok), "checked": "every deflate record OK; 64 outputs bit-exact vs the oracle "
            "(gzip, mtime 0); every inflate record success with checksum match; 64 round trips byte-compared"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["c4", "c5"], required=True)
    ap.add_argument("--scale", type=int, default=1)
    args = ap.parse_args()
    sdz.lib().sdz_set_timing(1)
    r = run_c4(args.scale) if args.config == "c4" else run_c5(args.scale)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
