#!/usr/bin/env python3
"""One-buffer facade calls of the reference's perf case (test/perf.html): inflate(paradiselost.deflate)
and deflate(paradiselost.txt, L1 / L6), one at a time, for a HIP-API / kernel trace of one call:
  rocprofv3 --runtime-trace --kernel-trace --stats -d gpurun_out/latb -- python3 tools/lat/lat_big.py
Prints the median milliseconds per call."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))
import sdz  # noqa: E402

g = os.path.join(ROOT, "tests", "golden")
c = open(os.path.join(g, "paradiselost.deflate"), "rb").read()
t = open(os.path.join(g, "paradiselost.txt"), "rb").read()
n = int(os.environ.get("LAT_N", "10"))
for name, f in (("inflate", lambda: sdz.inflate(c)), ("deflate_L1", lambda: sdz.deflate(t, {"level": 1})),
                ("deflate_L6", lambda: sdz.deflate(t, {"level": 6}))):
    f()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print("%s(paradiselost): median %.3f ms, min %.3f ms" % (name, 1e3 * ts[n // 2], 1e3 * ts[0]), flush=True)
