#!/bin/bash
# Round-3 second measurement call (through gpurun), after the deflate match changes: C3 deflate
# PMC passes -> profiles/r03_deflate_pmc.json (the bench's deflate traffic), the bench line and
# its kernel stats, then the C5 and C4 configs.  Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/deflate_prof
MODE=deflate STREAMS=65536 STEPS=1 PASSES="kt fetch write sq1 sq2" bash tools/profile_inflate.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof 1 gpurun_out/r03_deflate_pmc.json sdz::k_dfl,sdz::k_deflate,sdz::k_checksum > /dev/null || exit 1
cp gpurun_out/r03_deflate_pmc.json profiles/r03_deflate_pmc.json
mv gpurun_out/prof gpurun_out/deflate_prof
timeout -k 10 400 python3 bench.py > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || exit 1
cat gpurun_out/r03b_bench.json
rm -rf gpurun_out/bench_kt
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/bench_kt -o run --output-format csv -- \
    python3 bench.py > gpurun_out/r03b_bench_kt.json 2> gpurun_out/r03b_bench_kt.err || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c5 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c4 --scale 8 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 1
exit 0
