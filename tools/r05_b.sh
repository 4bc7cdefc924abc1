#!/bin/bash
# Round 5, second GPU call: the whole GPU suite on the shipped build, small-call latency, C2 /
# distinct / C3 timing, then the hot_epoch-inlined variants (bounds-checked first).  Every step
# writes to a file under gpurun_out/r05 as it goes; no development timing build (it hung the GPU
# in the first call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 700 $T tests -m gpu > $O/full_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc: $(tail -1 $O/full_gpu.log)"; [ $rc -eq 0 ] || grep -m12 -E "^FAILED|Error" $O/full_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 60 python3 tools/lat/lat_one.py > $O/lat.log 2>&1 || exit 1; cat $O/lat.log
for m in inflate distinct deflate; do
  timeout -k 10 200 python3 tools/run_c2.py --mode $m --steps 3 > $O/run_$m.log 2>&1 || exit 1; tail -1 $O/run_$m.log
done
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_hotchk.so SDZ_WDEC=1 timeout -k 10 150 $T -x -s tests/test_gpu_wdec.py -k "zlib_generated or many_small or oracle_generated" > $O/hotchk.log 2>&1
rc=$?; echo "hotchk rc=$rc: $(tail -1 $O/hotchk.log)"; grep -c IL_HOT_CHECK $O/hotchk.log; grep -m10 IL_HOT_CHECK $O/hotchk.log
[ $rc -eq 0 ] || exit $rc
grep -q IL_HOT_CHECK $O/hotchk.log && exit 0          # a check fired: read it before running unchecked
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_hotinl.so timeout -k 10 300 $T -x tests/test_gpu_wdec.py tests/test_gpu_lane.py > $O/hotinl.log 2>&1
rc=$?; echo "hotinl rc=$rc: $(tail -1 $O/hotinl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/hotinl.log; exit $rc; }
for m in inflate distinct; do
  SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_hotinl.so timeout -k 10 120 python3 tools/run_c2.py --mode $m --steps 3 > $O/hotinl_$m.log 2>&1 || exit 1; tail -1 $O/hotinl_$m.log
done
