#!/bin/bash
# C4 at a full per-GPU share: the cost model's threshold against forced ones, then a kernel
# trace of the default run (per-round decode/resolve times).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for sh in "" 0.05 0.1 0.25 0.5; do
  echo "== share ${sh:-model}"
  if [ -n "$sh" ]; then export SDZ_SPLIT_SHARE=$sh; else unset SDZ_SPLIT_SHARE; fi
  SDZ_SPLIT_DEBUG=1 timeout -k 10 200 python3 tools/run_configs.py --config c4 --scale 1 2>&1 | grep -E "sdz split|inflate:|kernel_ms" | cut -c1-260 || exit 1
done
unset SDZ_SPLIT_SHARE
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/c4kt" -o kt -- python3 "$GRAFT_REPO_ROOT/tools/run_configs.py" --config c4 --scale 1 > "$GRAFT_REPO_ROOT/gpurun_out/c4kt.log" 2>&1
