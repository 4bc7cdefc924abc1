#!/usr/bin/env python3
"""Single-buffer facade calls (C1 / perf.html's deflate(paradiselost)) for kernel traces:
  rocprofv3 --kernel-trace --stats -d gpurun_out/fprof -- python3 tools/facade_prof.py
Prints the wall time of each call; the trace attributes it to kernels."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))

import sdz  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    golden = os.path.join(ROOT, "tests", "golden")
    text = open(os.path.join(golden, "paradiselost.txt"), "rb").read()
    comp = open(os.path.join(golden, "paradiselost.deflate"), "rb").read()
    simple_c = open(os.path.join(golden, "simple.deflate"), "rb").read()
    simple_t = open(os.path.join(golden, "simple.txt"), "rb").read()
    cases = [("inflate_simple", lambda: sdz.inflate(simple_c)),
             ("deflate_simple", lambda: sdz.deflate(simple_t, {"level": 6})),
             ("inflate", lambda: sdz.inflate(comp))]
    for lv in (1, 4, 6, 9):
        cases.append(("deflate_L%d" % lv, lambda lv=lv: sdz.deflate(text, {"level": lv})))
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    for name, f in cases:
        if only and name not in only:
            continue
        f()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            f()
            ts.append(1e3 * (time.perf_counter() - t0))
        print("%-12s %s ms" % (name, " ".join("%.2f" % t for t in ts)), flush=True)


if __name__ == "__main__":
    main()
