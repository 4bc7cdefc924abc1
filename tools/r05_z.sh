#!/bin/bash
# Round 5: wave-decoder launch pairs queued two at a time (WD_PAIRS; libsdz_wdp1.so: one):
# inflate parity under the wave decoder and the default policy, the perf cases both ways.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_wdec.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_split.py \
    -k "not deflate and not Deflate" > $O/z_inf.log 2>&1
rc=$?; echo "inflate parity rc=$rc: $(tail -1 $O/z_inf.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/z_inf.log; exit $rc; }
for v in default wdp1 default wdp1; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"; SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 60 python3 tools/lat/lat_big.py | head -1 || exit 1
done
timeout -k 10 120 python3 tools/small_blocks_time.py 2>&1 | tail -3
