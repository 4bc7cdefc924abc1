#!/bin/bash
# C4 (1/8 share) at several round sizes (tokens per stream and round)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for t in 131072 524288 2097152; do
  echo "== round tokens $t"
  SDZ_ROUND_TOKENS=$t timeout -k 10 200 python3 tools/run_configs.py --config c4 --scale 8 2>&1 | grep -E "inflate:|kernel_ms" | cut -c1-260 || exit 1
done
