#!/bin/bash
# C4 (1/8 share) and C2 inflate for each library variant given (development aid)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for v in "$@"; do
  echo "== $v"
  SDZ_LIB=sd-zlib_amd/lib/$v timeout -k 10 200 python3 tools/run_configs.py --config c4 --scale 8 2>&1 | grep -E "inflate:|kernel_ms" | cut -c1-220 || exit 1
  SDZ_LIB=sd-zlib_amd/lib/$v timeout -k 10 120 python3 tools/run_c2.py --steps 2 2>&1 | grep "step 1" || exit 1
done
