#!/bin/bash
# Round 5: the resolve's serial tail (RS_SER: a group's last few tokens one at a time over the
# wave): inflate parity under all three decoder policies + streaming, then C2 / distinct for
# RS_SER 4 (default), 0 (off), 2, 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_lane.py tests/test_gpu_wdec.py tests/test_gpu_stream.py tests/test_gpu_split.py \
    tests/test_gpu_parity.py -k "not deflate and not Deflate" > $O/s_inf.log 2>&1
rc=$?; echo "inflate parity rc=$rc: $(tail -1 $O/s_inf.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/s_inf.log; exit $rc; }
for v in default ser0 ser2 ser8; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode inflate --steps 3 | tail -1 || exit 1
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode distinct --steps 3 | tail -1 || exit 1
done
