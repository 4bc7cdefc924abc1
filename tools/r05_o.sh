#!/bin/bash
# Round 5: deferred done events dropped after the host call's final wait; parse_wide's records
# taken from a 64-position register window: parity (host path, multi, streaming, deflate),
# latency, phase clocks, the trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_dict.py tests/test_gpu_multi.py tests/test_gpu_stream.py \
    tests/test_gpu_deflate_stream.py tests/test_gpu_deflate_fast.py > $O/o_par.log 2>&1
rc=$?; echo "parity rc=$rc: $(tail -1 $O/o_par.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/o_par.log; exit $rc; }
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
LAT_N=3 SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_dtprof.so timeout -k 10 60 python3 tools/lat/lat_one.py > $O/o_dtprof.log 2>&1
echo "dtprof rc=$?"; grep -m2 DT_PROF $O/o_dtprof.log; grep -m2 PW_PROF $O/o_dtprof.log
bash tools/lat/lat_trace.sh
