#!/usr/bin/env python3
"""Inflate time of a stream flushed every 256 bytes (~940 blocks), wave vs lane decoder, 1 and 64
streams (the wave decoder's alternation per block, and its lane hand-off after kWdLaneAfter)."""
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))
import sdz  # noqa: E402

data = open(os.path.join(ROOT, "tests", "golden", "paradiselost.txt"), "rb").read()[:240000]
c = zlib.compressobj(6)
comp = b"".join(c.compress(data[i:i + 256]) + c.flush(zlib.Z_SYNC_FLUSH) for i in range(0, len(data), 256)) + c.flush()
for mode, after in (("1", "16"), ("1", "100000000"), ("0", "16")):
    os.environ["SDZ_WDEC"] = mode
    os.environ["SDZ_WD_LANE_AFTER"] = after
    for n in (1, 64):
        best = 1e9
        for _ in range(4):
            t0 = time.perf_counter()
            g = sdz.inflate_batch([comp] * n, [len(data) + 4096] * n, sdz.FMT_CONTAINER)
            best = min(best, time.perf_counter() - t0)
        ok = all(x["status"] == "OK" and x["data"] == data for x in g)
        print("SDZ_WDEC=%s lane after %9s: streams %3d  %.2f ms  ok %s" % (mode, after, n, best * 1e3, ok), flush=True)
