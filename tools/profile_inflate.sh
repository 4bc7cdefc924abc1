#!/bin/bash
# Profiles the C2 inflate kernel on the GPU box (run through gpurun).
# Kernel trace/stats and each PMC group run as separate rocprofv3 passes
# (no --pmc together with trace domains).  Outputs under gpurun_out/prof/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
STREAMS=${STREAMS:-65536}
MODE=${MODE:-inflate}
step() {  # name, rocprof args...
    local name=$1; shift
    timeout -k 10 240 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- \
        python3 tools/run_c2.py --mode $MODE --streams $STREAMS --steps ${STEPS:-2} > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 $OUT/$name.log; fi
    return $rc
}
PASSES=${PASSES:-"kt fetch write sq1 sq2 tcc"}
for p in $PASSES; do
  case $p in
    kt) step kt --kernel-trace --stats || exit 1 ;;
    fetch) step pmc_fetch --pmc FETCH_SIZE || exit 1 ;;
    write) step pmc_write --pmc WRITE_SIZE || exit 1 ;;
    sq1) step pmc_sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1 ;;
    sq2) step pmc_sq2 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit 1 ;;
    sq3) step pmc_sq3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE || exit 1 ;;
    tcc) step pmc_tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum || exit 1 ;;
  esac
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt 2>&1 || true
exit 0
