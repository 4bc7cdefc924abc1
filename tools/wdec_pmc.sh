#!/bin/bash
# SQ counters of the wave decoder kernels on C2 (development aid; two separate --pmc passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/wpmc
M=${MODE:-inflate}
SDZ_WDEC=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    -d gpurun_out/wpmc/p1 -o run --output-format csv -- python3 tools/run_c2.py --mode $M --steps 1 > gpurun_out/wpmc/p1.log 2>&1 || exit 1
SDZ_WDEC=1 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
    -d gpurun_out/wpmc/p2 -o run --output-format csv -- python3 tools/run_c2.py --mode $M --steps 1 > gpurun_out/wpmc/p2.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
for f in glob.glob("gpurun_out/wpmc/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "wdec" in k or "wcold" in k or "resolve" in k:
            tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(tot.items()):
    print("%-26s %-22s %.4g" % (k, c, v))
PY
