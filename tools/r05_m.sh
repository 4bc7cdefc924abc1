#!/bin/bash
# Round 5: k_dfl_parse_wide run wave-uniform (PW_UNIFORM; libsdz_pwlane.so is lane 0), the tree
# kernel's overlapped prologue: deflate parity, small-call latency both ways, phase clocks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_fast.py tests/test_gpu_deflate_stream.py \
    tests/test_gpu_dict.py -k "deflate or Deflate or dict" > $O/m_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/m_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/m_dfl.log; exit $rc; }
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_pwlane.so timeout -k 10 60 python3 tools/lat/lat_one.py | tail -1 || exit 1
LAT_N=3 SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_dtprof.so timeout -k 10 60 python3 tools/lat/lat_one.py > $O/m_dtprof.log 2>&1
echo "dtprof rc=$?"; grep -m2 DT_PROF $O/m_dtprof.log; grep -m2 PW_PROF $O/m_dtprof.log
bash tools/lat/lat_trace.sh
