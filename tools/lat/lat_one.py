#!/usr/bin/env python3
"""C1-sized drop-in calls one at a time (inflate(simple.deflate), deflate(simple.txt)), for a
HIP-API / kernel trace of one call's timeline:
  rocprofv3 --runtime-trace --kernel-trace --stats -d gpurun_out/lat -- python3 tools/lat/lat_one.py
Prints the median microseconds per call."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))
import sdz  # noqa: E402

g = os.path.join(ROOT, "tests", "golden")
c = open(os.path.join(g, "simple.deflate"), "rb").read()
t = open(os.path.join(g, "simple.txt"), "rb").read()
n = int(os.environ.get("LAT_N", "100"))
for name, f, want in (("inflate", lambda: sdz.inflate(c), t), ("deflate", lambda: sdz.deflate(t, {"level": 6}), c)):
    assert f() == want
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print("%s(simple): median %.1f us, min %.1f us" % (name, 1e6 * ts[n // 2], 1e6 * ts[0]), flush=True)
