#!/bin/bash
# Round 5: k_dfl_match's first compare over 8 bytes (PM_W8, default build) -- deflate parity,
# C3 against the 4-byte form (libsdz_w4.so), and the long-compare counters (libsdz_cnt.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05d
O=gpurun_out/r05d
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py \
    -k "deflate or Deflate or dict" > $O/w8_dfl.log 2>&1
rc=$?; echo "w8 deflate parity rc=$rc: $(tail -1 $O/w8_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/w8_dfl.log; exit $rc; }
for v in default w4 default w4; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
done
echo "== counters (w8)"
SDZ_PHASE_TIMING=1 SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_cnt.so timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 1 2>&1 | tail -2
