#!/bin/bash
# Small-call timeline: tools/lat/lat_one.py (100 calls each of inflate(simple) / deflate(simple))
# under a HIP runtime + kernel trace; prints the per-API and per-kernel totals (rocprofv3 --stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05/lat_trace
rm -rf $O
LAT_N=100 timeout -k 10 120 rocprofv3 --runtime-trace --kernel-trace --stats -d $O -o run --output-format csv -- \
    python3 tools/lat/lat_one.py > gpurun_out/r05/lat_trace.log 2>&1
echo "lat trace rc=$?"; tail -2 gpurun_out/r05/lat_trace.log
for f in $O/*/run_hip_api_stats.csv $O/*/run_kernel_stats.csv; do
  [ -f "$f" ] && { echo "== $f"; head -25 "$f" | cut -d, -f1-4; }
done
exit 0
