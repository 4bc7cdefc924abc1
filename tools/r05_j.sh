#!/bin/bash
# Round 5: the small-call copy back by kernel (k_copy_back; SDZ_COPY_BACK=0 is the copy-engine
# copy), the parity suite through the host path, and the tree kernel's phase clocks (DT_PROF).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_dict.py tests/test_gpu_multi.py > $O/j_par.log 2>&1
rc=$?; echo "parity rc=$rc: $(tail -1 $O/j_par.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/j_par.log; exit $rc; }
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
SDZ_COPY_BACK=0 timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
LAT_N=3 SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_dtprof.so timeout -k 10 60 python3 tools/lat/lat_one.py > $O/j_dtprof.log 2>&1
echo "dtprof rc=$?"; grep -m3 DT_PROF $O/j_dtprof.log
T0=$(date +%s); timeout -k 10 200 python3 -u -c "
import sys; sys.path.insert(0,'sd-zlib_amd/python'); import sdz
d=open('tests/golden/paradiselost.txt','rb').read()
import time
for lv in (1,6,9):
    sdz.deflate(d,{'level':lv}); t=time.perf_counter(); sdz.deflate(d,{'level':lv}); print('paradiselost L%d %.2f ms'%(lv,1e3*(time.perf_counter()-t)))
" || exit 1
