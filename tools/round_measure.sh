#!/bin/bash
# Round-end measurement on the GPU box (run through gpurun):
#  1. rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE (+ SQ) passes of C2 -> HBM traffic JSON
#  2. bench.py (default config) with that traffic figure -> bench JSON line
#  3. rocprofv3 --kernel-trace --stats of the same bench command
# Outputs under gpurun_out/; the caller copies what is judged into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
STEPS=2 PASSES=${PASSES:-"kt fetch write sq1 sq2"} bash tools/profile_inflate.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof 2 gpurun_out/${TAG}_inflate_pmc.json > /dev/null || exit 1
cp gpurun_out/${TAG}_inflate_pmc.json profiles/${TAG}_inflate_pmc.json
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/bench_kt -o run --output-format csv -- \
    python3 bench.py > gpurun_out/${TAG}_bench_kt.json 2> gpurun_out/${TAG}_bench_kt.err || exit 1
exit 0
