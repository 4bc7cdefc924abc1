#!/bin/bash
# Development GPU call (through gpurun): the deflate parity tests (-k $K), then the C3 batch under
# rocprofv3 --kernel-trace --stats.  Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${K:-"4byte or deflate_record or deflate_all or deflate_edge or deflate_reference or full_paradise"}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TEST_LIMIT:-400} python3 -u -m pytest ${TEST_FILES:-tests/test_gpu_parity.py} -x -v --timeout 200 \
      --timeout-method thread -k "$K" > gpurun_out/pt_dev.log 2>&1
  rc=$?; tail -5 gpurun_out/pt_dev.log; [ $rc -ne 0 ] && exit $rc
fi
rm -rf gpurun_out/devkt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/devkt -o run -- \
    python3 tools/run_c2.py --mode deflate --steps ${STEPS:-2} --level ${LEVEL:-6} > gpurun_out/dev.log 2>&1
rc=$?; tail -4 gpurun_out/dev.log
[ $rc -ne 0 ] && exit $rc
if [ "${PMC:-0}" = 1 ]; then           # counter passes, each its own run (STEPS=1)
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    rm -rf gpurun_out/devpmc_$tag
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/devpmc_$tag -o run --output-format csv -- \
        python3 tools/run_c2.py --mode deflate --steps 1 --level ${LEVEL:-6} > gpurun_out/devpmc_$tag.log 2>&1 || exit 1
  done
fi
exit 0
