#!/bin/bash
# Round-5 closing measurement (after the k_dfl_match step work): the whole GPU suite + smoke + Node facade
# the bench line and its kernel trace on the final build.  Outputs under gpurun_out/r05e/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
LAT=1 NODE=1 bash tools/full_gpu.sh || exit 1
cp gpurun_out/full_gpu.log $O/
echo "== bench"
timeout -k 10 600 python3 bench.py > $O/r05e_bench.json 2> $O/r05e_bench.err || { tail -20 $O/r05e_bench.err; exit 1; }
cat $O/r05e_bench.json
echo "== bench kernel trace"
rm -rf $O/bench_kt
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $O/bench_kt -o run --output-format csv -- \
    python3 bench.py --node 0 --latency 0 --small-streams 0 > $O/r05e_bench_kt.json 2> $O/r05e_bench_kt.err || exit 1
exit 0
