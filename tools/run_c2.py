#!/usr/bin/env python3
"""Lightweight driver for profiling (no torch): runs the C2 inflate batch or the
C3 deflate batch K times through the C ABI and prints kernel times.
  rocprofv3 --kernel-trace --stats -- python3 tools/run_c2.py --mode inflate --steps 2
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))
sys.path.insert(0, ROOT)

import sdz  # noqa: E402
from bench import DeviceBatch, inflate_step, deflate_step, slice_offsets, fill_slices, inflate_distinct  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="inflate", choices=["inflate", "deflate", "distinct", "fast", "mixed"])
    ap.add_argument("--same", action="store_true", help="deflate: one slice in every stream")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--streams", type=int, default=65536)
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--slice", type=int, default=65536, help="deflate: bytes per stream")
    args = ap.parse_args()
    L = sdz.lib()
    L.sdz_set_timing(1)
    golden = os.path.join(ROOT, "tests", "golden")
    text = open(os.path.join(golden, "paradiselost.txt"), "rb").read()
    if args.mode == "inflate":
        comp = open(os.path.join(golden, "paradiselost.deflate"), "rb").read()
        b = DeviceBatch(sdz, comp, args.streams, len(text))
        for i in range(args.steps):
            split = []
            ms = inflate_step(sdz, b, split)
            print("inflate step %d: kernel %.3f ms (decode %.2f resolve %.2f), %.1f GB/s out"
                  % (i, ms, split[0][0], split[0][1], len(text) * args.streams / ms / 1e6), flush=True)
    elif args.mode == "distinct":
        # the bench's distinct-stream inflate leg: deflate n distinct slices (L6), inflate them
        import ctypes
        offs = slice_offsets(args.streams, len(text) - 65536)
        b = DeviceBatch(sdz, text[:65536], args.streams, int(L.sdz_deflate_bound(65536, 1, 0)))
        fill_slices(sdz, b, text, offs, 65536)
        deflate_step(sdz, b, args.level, 1)
        L.sdz_sync(None)
        drec = (sdz.DeflateRecord * args.streams).from_buffer_copy(
            b.d_rec.download(args.streams * ctypes.sizeof(sdz.DeflateRecord)))
        r, _ = inflate_distinct(sdz, L, b, drec, text, offs, 65536, args.steps, lambda: None, lambda x: x, 1)
        print("distinct inflate: kernel %.3f ms %s, %.1f GB/s out, parity %s"
              % (r["roofline"]["kernel_ms"], r["roofline"]["kernels_ms"],
                 r["config"]["bytes_out_per_gpu"] / r["roofline"]["kernel_ms"] / 1e6, r["parity"]), flush=True)
    elif args.mode == "mixed":
        # the bench's C4-shaped leg (one rank, every 8th stream of its LPT shard)
        from bench import mixed_leg
        r = mixed_leg(sdz, L, args.steps, 8, lambda: None, lambda x: x, 1, 0)
        print("mixed inflate: kernel %.3f ms %s, %.1f GB/s in+out, parity %s"
              % (r["kernel_ms"], r["roofline"]["kernels_ms"], r["roofline"]["achieved"], r["parity"]), flush=True)
        return
    elif args.mode == "fast":
        # the opt-in fast compressor on the C3 layout; validity checked with Python's zlib
        import ctypes
        import zlib
        offs = slice_offsets(args.streams, len(text) - 65536)
        b = DeviceBatch(sdz, text[:65536], args.streams, int(L.sdz_deflate_fast_bound(65536, 1, 0)))
        fill_slices(sdz, b, text, offs, 65536)
        for i in range(args.steps):
            in_off, in_len, out_off, out_cap = b.ptrs()
            rc = L.sdz_deflate_fast_batch_device(b.d_in.ptr, in_off, in_len, b.d_out.ptr, out_off, out_cap,
                                                 b.d_rec.ptr, b.n, 1, None, 0, 0, None)
            if rc:
                raise RuntimeError(L.sdz_last_error().decode())
            ms = L.sdz_last_kernel_ms()
            recs = (sdz.DeflateRecord * args.streams).from_buffer_copy(
                b.d_rec.download(args.streams * ctypes.sizeof(sdz.DeflateRecord)))
            tot = sum(r.out_len for r in recs)
            ok = all(r.status == 0 for r in recs)
            for k in range(0, args.streams, max(1, args.streams // 64)):
                data = b.d_out.download(recs[k].out_len, k * b.out_stride)
                ok = ok and zlib.decompress(data) == text[offs[k]:offs[k] + 65536]
            print("fast deflate step %d: kernel %.3f ms, %.2f GB/s in, %.2f GB/s out, ratio %.3f, valid %s"
                  % (i, ms, 65536 * args.streams / ms / 1e6, tot / ms / 1e6, tot / (65536 * args.streams), ok),
                  flush=True)
    else:
        # the bench's C3 layout: distinct slices of paradiselost.txt at xorshift64 offsets
        # (identical streams would run the serial parse without any lane divergence)
        sl = args.slice
        b = DeviceBatch(sdz, text[:sl], args.streams, int(L.sdz_deflate_bound(sl, 1, 0)))
        if not args.same:
            fill_slices(sdz, b, text, slice_offsets(args.streams, len(text) - sl), sl)
        for i in range(args.steps):
            ms = deflate_step(sdz, b, args.level, 1)
            print("deflate step %d: kernel %.3f ms, %.2f GB/s in" % (i, ms, sl * args.streams / ms / 1e6),
                  flush=True)
    b.free()


if __name__ == "__main__":
    main()
