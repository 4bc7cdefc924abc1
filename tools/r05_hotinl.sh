#!/bin/bash
# Round 5, first GPU call: (1) the lane-decoder parity suite (SDZ_WDEC=0) and the split tests;
# (2) the hot_epoch-inlined variant with bounds checks (IL_HOT_CHECK: an out-of-bounds access is
# printed and skipped, not executed) on the test that faulted in round 4; (3) the inlined variant
# with the idle-lane fix alone; (4) C2 / distinct timing of the shipped build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_lane.py tests/test_gpu_split.py > $O/lane_tests.log 2>&1
rc=$?; echo "lane+split rc=$rc: $(tail -1 $O/lane_tests.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/lane_tests.log; exit $rc; }
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_hotchk.so SDZ_WDEC=1 timeout -k 10 200 $T -s tests/test_gpu_wdec.py -k "zlib_generated or many_small or oracle_generated" > $O/hotchk.log 2>&1
rc=$?; echo "hotchk rc=$rc: $(tail -1 $O/hotchk.log)"; grep -c IL_HOT_CHECK $O/hotchk.log; grep -m10 IL_HOT_CHECK $O/hotchk.log
[ $rc -eq 0 ] || exit $rc
grep -q IL_HOT_CHECK $O/hotchk.log && exit 0          # a check fired: read it before running unchecked
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_hotinl.so timeout -k 10 300 $T tests/test_gpu_wdec.py tests/test_gpu_lane.py > $O/hotinl.log 2>&1
rc=$?; echo "hotinl rc=$rc: $(tail -1 $O/hotinl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/hotinl.log; exit $rc; }
for lib in libsdz.so libsdz_hotinl.so; do
  echo "== $lib"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode inflate --steps 3 | tail -2 || exit 1
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode distinct --steps 3 | tail -1 || exit 1
done
