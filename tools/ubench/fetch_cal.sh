#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (tools/ubench/fetch_cal.hip) on the GPU box: separate
# counter passes, then counter bytes / known bytes per kernel -> gpurun_out/fetch_cal.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fcal
B=tools/ubench/fetch_cal
[ -x $B ] || hipcc --offload-arch=gfx950 -O3 -o $B tools/ubench/fetch_cal.hip || exit 1
timeout -k 10 60 ./$B time > gpurun_out/fcal/time.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fcal/f -o run --output-format csv -- ./$B > gpurun_out/fcal/f.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/fcal/w -o run --output-format csv -- ./$B > gpurun_out/fcal/w.log 2>&1 || exit 1
python3 - <<'PY' | tee gpurun_out/fetch_cal.txt
import csv, glob
import json
known = {"k_stream16": 2 << 30, "k_scatter1": (2 << 30) // 128 * 128, "k_scatter8": (2 << 30) // 128 * 128,
         "k_scatter2": (2 << 30) // 128 * 128,
         "k_lane8": 2 << 30, "k_lane16": 2 << 30, "k_store8": 2 << 30}
res = {}
for c, d in (("FETCH_SIZE", "f"), ("WRITE_SIZE", "w")):
    for path in glob.glob("gpurun_out/fcal/%s/**/*counter_collection.csv" % d, recursive=True):
        tot = {}
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != c:
                continue
            k = r["Kernel_Name"].split("(")[0]
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"]) * 1024
        for k, v in sorted(tot.items()):
            print("%s %-12s %.4g B  /known(lines x 128 B or bytes) = %.3f" % (c, k, v, v / known.get(k, 1)))
            res.setdefault(c, {})[k.replace("k_", "")] = v / known.get(k, 1)
rates = {}
for l in open("gpurun_out/fcal/time.txt"):
    f = l.split()
    if f and f[0] == "READ":
        rates[f[1]] = float(f[4])
        print("read rate %-9s %.1f GB/s (known bytes / best of 5)" % (f[1], rates[f[1]]))
json.dump({"counter_bytes_over_known": res, "read_GBps": rates, "note": "FETCH_SIZE/WRITE_SIZE x 1024 over the bytes each kernel "
           "touches once (scatter: distinct 128-B lines x 128 B); tools/ubench/fetch_cal.hip"},
          open("gpurun_out/fetch_cal.json", "w"), indent=1)
PY
