#!/bin/bash
# Everything a round's judged numbers come from, in one GPU call (run through gpurun):
#  1. deflate (C3) kernel trace (its 65 Ki slice copies under --pmc broke the queue: no PMC pass) -> gpurun_out/prof_dfl/
#  2. tools/round_measure.sh: inflate (C2) profile passes, HBM traffic, bench line, bench
#     under rocprofv3 --kernel-trace --stats            -> gpurun_out/
#  3. BASELINE configs C5 (full per-GPU share) and C4 (1/8 share) -> gpurun_out/c5.json, c4.json
# Each GPU step has its own time limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/prof_dfl
MODE=deflate STREAMS=65536 STEPS=1 PASSES="kt" bash tools/profile_inflate.sh || exit 1
mv gpurun_out/prof gpurun_out/prof_dfl
TAG=${TAG:-r01} bash tools/round_measure.sh || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c5 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c4 --scale 8 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 1
exit 0
