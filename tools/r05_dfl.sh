#!/bin/bash
# Round 5: the last-position searches in k_dfl_match (parity, then C3 timing against the all-HBM
# tail, SDZ_TAIL_HBM=1) and the long-compare test behind one branch (PM_MORE_IF; variant lib
# libsdz_moreoff.so is the old loop).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py -k "deflate" > $O/dfl_tests.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/dfl_tests.log)"; [ $rc -eq 0 ] || grep -m8 -E "Error|assert|FAIL" $O/dfl_tests.log
[ $rc -le 1 ] || exit $rc
for v in default tailhbm moreoff; do
  lib=libsdz.so; env=""
  [ $v = tailhbm ] && env="SDZ_TAIL_HBM=1"
  [ $v = moreoff ] && lib=libsdz_moreoff.so
  [ -f sd-zlib_amd/lib/$lib ] || continue
  echo "== $v"
  env $env SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -2 || exit 1
done
