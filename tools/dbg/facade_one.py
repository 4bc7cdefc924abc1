#!/usr/bin/env python3
"""inflate(paradiselost.deflate) through the facade, 20 calls (for a kernel trace of one call's timeline)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))
import sdz  # noqa: E402

comp = open(os.path.join(ROOT, "tests", "golden", "paradiselost.deflate"), "rb").read()
text = open(os.path.join(ROOT, "tests", "golden", "paradiselost.txt"), "rb").read()
for i in range(20):
    t0 = time.perf_counter()
    out = sdz.inflate(comp)
    dt = time.perf_counter() - t0
    if i >= 17:
        print("call %d: %.3f ms ok %s" % (i, dt * 1e3, out == text), flush=True)
