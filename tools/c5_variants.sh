#!/bin/bash
# C5 (gzip L9 round trip) inflate/deflate times for each library in LIBS (development aid)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for lib in ${LIBS:-libsdz.so}; do
  echo "== $lib"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 300 python3 tools/run_configs.py --config c5 > gpurun_out/c5_$lib.json 2>/dev/null || exit 1
  grep -o '"inflate_kernel_ms[^,]*\|"parity[^,]*' gpurun_out/c5_$lib.json
done
