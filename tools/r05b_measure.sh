#!/bin/bash
# Round-5 second measurement (after the tree kernel, the small-call and marker changes): C3 deflate
# kernel stats + PMC passes (-> profiles/r05_deflate_pmc.json), the bench line and its kernel
# trace, C4 / C5.  The inflate kernels did not change since tools/r05_measure.sh: the C2 counters
# (profiles/r05_inflate_pmc.json) stand.  Outputs under gpurun_out/r05b/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
step() { echo "== $*"; }
step C3 deflate counters
rm -rf gpurun_out/prof
MODE=deflate STREAMS=65536 STEPS=1 PASSES="kt fetch write sq1 sq2" bash tools/profile_inflate.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof 1 $O/r05_deflate_pmc.json sdz::k_dfl,sdz::k_deflate,sdz::k_checksum profiles/r04_fetch_cal.json > /dev/null || exit 1
rm -rf $O/deflate_pmc && mv gpurun_out/prof $O/deflate_pmc
cp $O/r05_deflate_pmc.json profiles/
step bench
timeout -k 10 600 python3 bench.py > $O/r05b_bench.json 2> $O/r05b_bench.err || { tail -20 $O/r05b_bench.err; exit 1; }
cat $O/r05b_bench.json
step bench kernel trace
rm -rf $O/bench_kt
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $O/bench_kt -o run --output-format csv -- \
    python3 bench.py --node 0 --latency 0 --small-streams 0 > $O/r05b_bench_kt.json 2> $O/r05b_bench_kt.err || exit 1
step configs
timeout -k 10 300 python3 tools/run_configs.py --config c5 > $O/c5.json 2> $O/c5.err || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c4 --scale 8 > $O/c4.json 2> $O/c4.err || exit 1
tail -n 3 $O/c5.json $O/c4.json
exit 0
