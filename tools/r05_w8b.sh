#!/bin/bash
# Round 5: the shipped k_dfl_match (8-byte first compare, refill at 12 idle lanes): deflate
# parity, C3 kernel stats, and one counter pass (LDS instructions and bank conflicts).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05d
O=gpurun_out/r05d
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py \
    -k "deflate or Deflate or dict" > $O/w8b_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/w8b_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/w8b_dfl.log; exit $rc; }
rm -rf $O/kt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 tools/run_c2.py --mode deflate --steps 3 > $O/kt.log 2>&1
rc=$?; tail -2 $O/kt.log; [ $rc -eq 0 ] || exit $rc
rm -rf $O/pmc_sq
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT \
    -d $O/pmc_sq -o run --output-format csv -- python3 tools/run_c2.py --mode deflate --steps 1 > $O/pmc_sq.log 2>&1
rc=$?; tail -1 $O/pmc_sq.log; exit $rc
