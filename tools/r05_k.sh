#!/bin/bash
# Round 5: k_dfl_trees with the heap in registers and scan_tree / send_tree over the wave:
# deflate parity, small-call latency, C3 timing (against the lane-0 kernel, libsdz_dtlane.so),
# phase clocks (DT_PROF: tree kernel and parse_wide).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_fast.py tests/test_gpu_deflate_stream.py \
    tests/test_gpu_dict.py -k "deflate or Deflate or dict" > $O/k_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/k_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/k_dfl.log; exit $rc; }
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
for v in default dtlane; do
  lib=libsdz.so; [ $v = dtlane ] && lib=libsdz_dtlane.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
done
LAT_N=3 SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_dtprof.so timeout -k 10 60 python3 tools/lat/lat_one.py > $O/k_dtprof.log 2>&1
echo "dtprof rc=$?"; grep -m2 DT_PROF $O/k_dtprof.log; grep -m2 PW_PROF $O/k_dtprof.log
timeout -k 10 200 python3 -u -c "
import sys; sys.path.insert(0,'sd-zlib_amd/python'); import sdz
d=open('tests/golden/paradiselost.txt','rb').read()
import time
for lv in (1,6,9):
    sdz.deflate(d,{'level':lv}); t=time.perf_counter(); sdz.deflate(d,{'level':lv}); print('paradiselost L%d %.2f ms'%(lv,1e3*(time.perf_counter()-t)))
" || exit 1
