#!/bin/bash
# Round 5: the wave-cooperative k_dfl_trees (DT_WAVE=1): deflate parity, small-call latency,
# C3 timing against the lane-0 tree kernel (libsdz_dtlane.so, DT_WAVE=0), the small-call trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_fast.py tests/test_gpu_deflate_stream.py \
    tests/test_gpu_dict.py -k "deflate or Deflate or dict" > $O/i_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/i_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/i_dfl.log; exit $rc; }
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
for v in default dtlane; do
  lib=libsdz.so; [ $v = dtlane ] && lib=libsdz_dtlane.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
done
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_dtlane.so timeout -k 10 60 python3 tools/lat/lat_one.py | tail -1 || exit 1
bash tools/lat/lat_trace.sh
