#!/bin/bash
# timeline of the one-buffer perf-case calls (tools/lat/lat_big.py) under a HIP runtime + kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05/latb_trace
rm -rf $O
timeout -k 10 60 python3 tools/lat/lat_big.py || exit 1
LAT_N=5 timeout -k 10 180 rocprofv3 --runtime-trace --kernel-trace --memory-copy-trace --stats -d $O -o run --output-format csv -- \
    python3 tools/lat/lat_big.py > gpurun_out/r05/latb_trace.log 2>&1
echo "latb trace rc=$?"; tail -3 gpurun_out/r05/latb_trace.log
exit 0
