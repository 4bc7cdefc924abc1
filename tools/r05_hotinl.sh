#!/bin/bash
# Round 5, first GPU call, the riskiest step last:
#  (1) the lane-decoder parity suite (SDZ_WDEC=0), the split tests, the multi-GPU tests;
#  (2) small-call latency (tools/lat/lat_one.py), with and without the serial small-deflate path;
#  (3) C2 / distinct timing of the shipped build;
#  (4) tools/r05_dfl.sh (deflate parity + C3 timings), tools/r05_phase.sh (inflate phase clocks);
#  (5) the hot_epoch-inlined variant with bounds checks (IL_HOT_CHECK: an out-of-bounds access is
#      printed and skipped, not executed) on the test that faulted in round 4, then the inlined
#      variant with the idle-lane fix alone.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_lane.py tests/test_gpu_split.py tests/test_gpu_multi.py > $O/lane_tests.log 2>&1
rc=$?; echo "lane+split+multi rc=$rc: $(tail -1 $O/lane_tests.log)"; [ $rc -eq 0 ] || grep -m8 -E "Error|assert|FAIL" $O/lane_tests.log
[ $rc -le 1 ] || exit $rc                              # (1: failed tests, read later; anything else ends here)
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
SDZ_DEFLATE_SMALL=0 timeout -k 10 60 python3 tools/lat/lat_one.py | tail -1 || exit 1
timeout -k 10 120 python3 tools/run_c2.py --mode inflate --steps 3 | tail -2 || exit 1
timeout -k 10 120 python3 tools/run_c2.py --mode distinct --steps 3 | tail -1 || exit 1
bash tools/r05_dfl.sh || exit 1
bash tools/r05_phase.sh || exit 1
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_hotchk.so SDZ_WDEC=1 timeout -k 10 200 $T -x -s tests/test_gpu_wdec.py -k "zlib_generated or many_small or oracle_generated" > $O/hotchk.log 2>&1
rc=$?; echo "hotchk rc=$rc: $(tail -1 $O/hotchk.log)"; grep -c IL_HOT_CHECK $O/hotchk.log; grep -m10 IL_HOT_CHECK $O/hotchk.log
[ $rc -eq 0 ] || exit $rc
grep -q IL_HOT_CHECK $O/hotchk.log && exit 0          # a check fired: read it before running unchecked
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_hotinl.so timeout -k 10 300 $T -x tests/test_gpu_wdec.py tests/test_gpu_lane.py > $O/hotinl.log 2>&1
rc=$?; echo "hotinl rc=$rc: $(tail -1 $O/hotinl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/hotinl.log; exit $rc; }
echo "== hotinl timing"
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_hotinl.so timeout -k 10 120 python3 tools/run_c2.py --mode inflate --steps 3 | tail -2 || exit 1
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_hotinl.so timeout -k 10 120 python3 tools/run_c2.py --mode distinct --steps 3 | tail -1 || exit 1
