#!/bin/bash
# Round-3 measurement call (through gpurun): C2 PMC passes + bench line + bench kernel stats
# (tools/round_measure.sh), then the C5 and C4 configs.  Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r03 bash tools/round_measure.sh || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c5 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c4 --scale 8 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 1
exit 0
