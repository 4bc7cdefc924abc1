#!/usr/bin/env python3
"""One configuration of tools/small_blocks_time.py (argv: SDZ_WDEC value, streams), for a kernel trace."""
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))
os.environ["SDZ_WDEC"] = sys.argv[1]
import sdz  # noqa: E402

n = int(sys.argv[2])
data = open(os.path.join(ROOT, "tests", "golden", "paradiselost.txt"), "rb").read()[:240000]
c = zlib.compressobj(6)
comp = b"".join(c.compress(data[i:i + 256]) + c.flush(zlib.Z_SYNC_FLUSH) for i in range(0, len(data), 256)) + c.flush()
for _ in range(3):
    t0 = time.perf_counter()
    g = sdz.inflate_batch([comp] * n, [len(data) + 4096] * n, sdz.FMT_CONTAINER)
    print("%.2f ms" % ((time.perf_counter() - t0) * 1e3), all(x["data"] == data for x in g), flush=True)
