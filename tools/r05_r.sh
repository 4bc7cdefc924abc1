#!/bin/bash
# Round 5: k_dfl_encode rows with a DPP scan and double-buffered stage / sums (EN_V2; the
# libsdz_env1.so variant is the old loop): deflate parity, C3 both ways.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_fast.py tests/test_gpu_deflate_stream.py \
    tests/test_gpu_dict.py -k "deflate or Deflate or dict" > $O/r_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/r_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/r_dfl.log; exit $rc; }
for v in default env1 default env1; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
done
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
