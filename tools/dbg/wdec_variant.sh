#!/bin/bash
# a wave-decoder variant library (make variant V=...) against the default: wdec-forced parity
# tests, one facade call, 1,024 and 16,384 paradiselost copies, distinct 16,384
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp
V=${V:-r11}
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_$V.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wdec.py ${TESTS:-} > gpurun_out/wvar_tests.log 2>&1 || { tail -20 gpurun_out/wvar_tests.log; exit 1; }
tail -1 gpurun_out/wvar_tests.log
for lib in libsdz.so libsdz_$V.so; do
  echo "== $lib"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 60 python3 tools/dbg/facade_one.py | tail -1 || exit 1
  for n in 1024 16384; do
    SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib SDZ_WDEC=1 timeout -k 10 60 python3 tools/run_c2.py --mode inflate --streams $n --steps 2 | tail -1 || exit 1
  done
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib SDZ_WDEC=1 timeout -k 10 60 python3 tools/run_c2.py --mode distinct --streams 16384 --steps 2 | tail -1 || exit 1
  if [ -n "${LANE:-}" ]; then
    SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode inflate --steps 2 | tail -1 || exit 1
    SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode distinct --steps 2 | tail -1 || exit 1
  fi
done
