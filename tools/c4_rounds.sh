#!/bin/bash
# C4 (1/8 share) inflate time against the per-round token budget (development aid)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for t in ${TOKENS:-131072 524288 2097152}; do
  echo "== SDZ_ROUND_TOKENS=$t"
  SDZ_ROUND_TOKENS=$t timeout -k 10 300 python3 tools/run_configs.py --config c4 --scale 8 > gpurun_out/c4_$t.json 2>/dev/null || exit 1
  grep -o '"kernel_ms[^,]*\|"parity[^,]*' gpurun_out/c4_$t.json
done
