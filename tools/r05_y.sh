#!/bin/bash
# Round 5: k_lz_blocks with one reduction pass per window and 1,024 threads for few streams:
# deflate parity, perf cases; then the wave decoder's cold kernel phase clocks (IL_PROF variant,
# printf from stream 0) on one inflate(paradiselost).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py \
    -k "deflate or Deflate or dict" > $O/y_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/y_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/y_dfl.log; exit $rc; }
timeout -k 10 60 python3 tools/lat/lat_big.py || exit 1
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_ilprof.so timeout -k 10 60 python3 -c "
import sys; sys.path.insert(0,'sd-zlib_amd/python'); import sdz
c=open('tests/golden/paradiselost.deflate','rb').read(); t=open('tests/golden/paradiselost.txt','rb').read()
assert sdz.inflate(c)==t; assert sdz.inflate(c)==t; print('ilprof ok')
" > $O/y_ilprof.log 2>&1
echo "ilprof rc=$?"; grep -c WC_PROF $O/y_ilprof.log; grep WC_PROF $O/y_ilprof.log | tail -16
