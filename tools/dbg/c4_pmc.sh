#!/bin/bash
# SQ counter passes over C4 (1/8 share), one rocprofv3 --pmc run each (gpurun)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/c4pmc
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $OUT/p1 -o run --output-format csv -- python3 tools/run_configs.py --config c4 --scale 8 > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -d $OUT/p2 -o run --output-format csv -- python3 tools/run_configs.py --config c4 --scale 8 > $OUT/p2.log 2>&1 || exit 1
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
