#!/bin/bash
# Round 5: deflate(simple) / inflate(simple) single-call latency, the round-5c build's k_deflate
# (libsdz_old.so) against the current one, then each under a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05e
for v in old default old default; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"; SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib LAT_N=400 timeout -k 10 120 python3 tools/lat/lat_one.py || exit 1
done
for v in old default; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  rm -rf gpurun_out/r05e/lat_$v
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib LAT_N=100 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05e/lat_$v -o run \
      --output-format csv -- python3 tools/lat/lat_one.py > gpurun_out/r05e/lat_$v.log 2>&1 || exit 1
  f=$(ls gpurun_out/r05e/lat_$v/*/run_kernel_stats.csv); echo "== kernels $v"; head -20 $f | cut -d, -f1-4
done
