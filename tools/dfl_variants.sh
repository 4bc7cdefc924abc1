#!/bin/bash
# deflate parity (pytest -k deflate) and C3 timing (16 Ki streams) for each library in LIBS
# (development aid, run through gpurun); the first failure ends it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for lib in ${LIBS:-libsdz.so}; do
  echo "== $lib"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 300 python3 -m pytest tests -m gpu -x -q -k "deflate" > gpurun_out/pt_$lib.log 2>&1
  rc=$?; tail -1 gpurun_out/pt_$lib.log; [ $rc -ne 0 ] && exit $rc
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode deflate --streams ${STREAMS:-16384} --steps 2 2>&1 | grep -i "step\|error" || exit 1
done
