#!/bin/bash
# lane-decoder variant libraries (make variant V=...) on C2 and the distinct leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp
for lib in libsdz.so ${VARIANTS-libsdz_s0.so libsdz_s2.so}; do
  for m in inflate distinct; do
    r=$(SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode $m --steps 3 | tail -1) || exit 1
    echo "$lib $m: $r"
  done
done
