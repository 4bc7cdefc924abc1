#!/usr/bin/env python3
"""Streaming facade timings: Inflater.append / Deflater.append with large chunks (the drop-in's
incremental classes), next to the one-shot calls."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python"))

import sdz  # noqa: E402


def t(f, k=3):
    f()
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        f()
        ts.append(1e3 * (time.perf_counter() - t0))
    return " ".join("%.2f" % x for x in ts)


def main():
    golden = os.path.join(ROOT, "tests", "golden")
    text = open(os.path.join(golden, "paradiselost.txt"), "rb").read()
    comp = open(os.path.join(golden, "paradiselost.deflate"), "rb").read()

    def inf_whole():
        i = sdz.Inflater()
        i.append(comp)
        i.finish()

    def inf_64k():
        i = sdz.Inflater()
        for o in range(0, len(comp), 65536):
            i.append(comp[o:o + 65536])
        i.finish()

    def def_whole():
        d = sdz.Deflater({"level": 6})
        d.append(text)
        d.finish()

    print("inflate()            %s ms" % t(lambda: sdz.inflate(comp)), flush=True)
    print("Inflater one append  %s ms" % t(inf_whole), flush=True)
    print("Inflater 64K appends %s ms" % t(inf_64k), flush=True)
    print("deflate() L6         %s ms" % t(lambda: sdz.deflate(text, {"level": 6})), flush=True)
    print("Deflater one append  %s ms" % t(def_whole, 1), flush=True)
    big = text * 10

    def def_stream():
        d = sdz.Deflater({"level": 6})
        for o in range(0, len(big), 65536):
            d.append(big[o:o + 65536])
        d.finish()
    print("Deflater 4.7 MB in 64 KiB appends %s ms" % t(def_stream, 1), flush=True)
    print("deflate() 4.7 MB     %s ms" % t(lambda: sdz.deflate(big, {"level": 6}), 2), flush=True)


if __name__ == "__main__":
    main()
