#!/usr/bin/env python3
"""HBM traffic per inflate launch from rocprofv3 PMC passes (tools/profile_inflate.sh).

One launch of sdz_inflate_batch_device = k_inflate_decode + k_inflate_resolve
(per round) + k_inflate_finalize.  Per MI355X_MICROARCH.md (HBM/rocprofv3):
FETCH_SIZE and WRITE_SIZE come from separate passes, are in KiB, and on gfx950
FETCH_SIZE reports half of the bytes of wide reads -- doubled here.
Usage: pmc_traffic.py <prof dir> <steps> <out.json> [kernel prefixes, comma-separated]
(default sdz::k_inflate; the deflate leg: sdz::k_dfl,sdz::k_deflate,sdz::k_checksum)
"""
import collections
import csv
import json
import os
import sys


PREFIXES = ("sdz::k_inflate",)


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0]
        if not k.startswith(PREFIXES):
            continue
        tot[k] += float(r["Counter_Value"])
        n[k] += 1
    return tot, n


def main():
    global PREFIXES
    root, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    if len(sys.argv) > 4:
        PREFIXES = tuple(sys.argv[4].split(","))
    f, nf = per_kernel(os.path.join(root, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w, nw = per_kernel(os.path.join(root, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    kernels = sorted(set(f) | set(w))
    rows = {}
    total = 0.0
    for k in kernels:
        fb = 2 * 1024 * f.get(k, 0.0) / steps            # per launch (all rounds), gfx950 x2
        wb = 1024 * w.get(k, 0.0) / steps
        rows[k] = {"fetch_bytes": fb, "write_bytes": wb, "dispatches_per_launch": nf.get(k, 0) / steps}
        total += fb + wb
    res = {"hbm_bytes_per_launch": total, "per_kernel": rows,
           "note": "FETCH_SIZE doubled (gfx950 reports half of wide reads); KiB -> bytes"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
