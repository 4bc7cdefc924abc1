#!/bin/bash
# Round 5: k_dfl_match refill without a divergent region (PM_SELFILL: every lane reads, selects) --
# deflate parity, then C3 against the branchy refill (libsdz_nosf.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05d
O=gpurun_out/r05d
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py \
    -k "deflate or Deflate or dict" > $O/sf_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/sf_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/sf_dfl.log; exit $rc; }
for v in default nosf default nosf; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
done
