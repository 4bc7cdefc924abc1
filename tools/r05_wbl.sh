#!/bin/bash
# Round 5: the byte-at-best filter after the 8-byte compare (PM_WBLATE, default build) -- deflate
# parity, C3 against the filter read for every candidate (libsdz_wbe.so), long-compare counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05d
O=gpurun_out/r05d
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py \
    -k "deflate or Deflate or dict" > $O/wbl_dfl.log 2>&1
rc=$?; echo "wblate deflate parity rc=$rc: $(tail -1 $O/wbl_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/wbl_dfl.log; exit $rc; }
for v in default wbe default wbe; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
done
echo "== counters (wblate)"
SDZ_PHASE_TIMING=1 SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_cnt.so timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 1 2>&1 | tail -2
