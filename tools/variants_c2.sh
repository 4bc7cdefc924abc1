#!/bin/bash
# C2 + distinct-stream inflate timing for each library variant given (run through gpurun):
#   bash tools/variants_c2.sh libsdz.so libsdz_foo.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  echo "== $v"
  SDZ_LIB=sd-zlib_amd/lib/$v timeout -k 10 120 python3 tools/run_c2.py --steps 2 || exit 1
  SDZ_LIB=sd-zlib_amd/lib/$v timeout -k 10 200 python3 tools/run_c2.py --mode distinct --steps 2 || exit 1
done
