#!/bin/bash
# Round 5: k_dfl_match with the byte-at-best filter read only where best >= 4 (PM_WBSKIP,
# libsdz_wbskip.so): its deflate parity, then C3 against the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_wbskip.so timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py \
    tests/test_gpu_dict.py -k "deflate or Deflate or dict" > $O/p_dfl.log 2>&1
rc=$?; echo "wbskip deflate parity rc=$rc: $(tail -1 $O/p_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/p_dfl.log; exit $rc; }
for v in default wbskip default wbskip; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
done
