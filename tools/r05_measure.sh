#!/bin/bash
# Round-5 measurement call (through gpurun): FETCH/WRITE_SIZE calibration, C2 inflate and C3 deflate
# kernel stats + PMC passes of the same build the bench times (-> profiles/r05_*_pmc.json, read by
# bench.py), the bench line and its kernel trace, then the C4 / C5 configs.  Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
step() { echo "== $*"; }
# the FETCH_SIZE / WRITE_SIZE calibration is the hardware's (round 4: profiles/r04_fetch_cal.json)
cp profiles/r04_fetch_cal.json gpurun_out/r05/r05_fetch_cal.json
step C2 inflate counters
rm -rf gpurun_out/prof
MODE=inflate STREAMS=65536 STEPS=2 PASSES="kt fetch write sq1 sq2" bash tools/profile_inflate.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof 2 gpurun_out/r05/r05_inflate_pmc.json sdz::k_inflate gpurun_out/r05/r05_fetch_cal.json > /dev/null || exit 1
rm -rf gpurun_out/r05/c2_pmc && mv gpurun_out/prof gpurun_out/r05/c2_pmc
step C3 deflate counters
MODE=deflate STREAMS=65536 STEPS=1 PASSES="kt fetch write sq1 sq2" bash tools/profile_inflate.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof 1 gpurun_out/r05/r05_deflate_pmc.json sdz::k_dfl,sdz::k_deflate,sdz::k_checksum gpurun_out/r05/r05_fetch_cal.json > /dev/null || exit 1
rm -rf gpurun_out/r05/deflate_pmc && mv gpurun_out/prof gpurun_out/r05/deflate_pmc
# the bench reads the latest profiles/rNN_*_pmc.json: stage them in the tree for this run's bench
cp gpurun_out/r05/r05_inflate_pmc.json gpurun_out/r05/r05_deflate_pmc.json profiles/
step bench
timeout -k 10 600 python3 bench.py > gpurun_out/r05/r05_bench.json 2> gpurun_out/r05/r05_bench.err || { tail -20 gpurun_out/r05/r05_bench.err; exit 1; }
cat gpurun_out/r05/r05_bench.json
step bench kernel trace
rm -rf gpurun_out/r05/bench_kt
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/r05/bench_kt -o run --output-format csv -- \
    python3 bench.py --node 0 --latency 0 --small-streams 0 > gpurun_out/r05/r05_bench_kt.json 2> gpurun_out/r05/r05_bench_kt.err || exit 1
step configs
timeout -k 10 300 python3 tools/run_configs.py --config c5 > gpurun_out/r05/c5.json 2> gpurun_out/r05/c5.err || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c4 --scale 8 > gpurun_out/r05/c4.json 2> gpurun_out/r05/c4.err || exit 1
tail -n 3 gpurun_out/r05/c5.json gpurun_out/r05/c4.json
exit 0
