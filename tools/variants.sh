#!/bin/bash
# time C2 inflate under several libsdz builds (SDZ_LIB), development aid
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in "$@"; do
  echo "== $lib"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode inflate --streams ${STREAMS:-65536} --steps 2 || exit 1
done
