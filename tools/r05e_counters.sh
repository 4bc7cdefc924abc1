#!/bin/bash
# Round-5 measurement after the k_dfl_match step work: C3 deflate kernel stats + PMC passes
# (-> r05_deflate_pmc.json, copied to profiles/ by hand), C5 and C4.  Outputs under gpurun_out/r05e/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
step() { echo "== $*"; }
step C3 deflate counters
rm -rf gpurun_out/prof
MODE=deflate STREAMS=65536 STEPS=1 PASSES="kt fetch write sq1 sq2" bash tools/profile_inflate.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof 1 $O/r05_deflate_pmc.json sdz::k_dfl,sdz::k_deflate,sdz::k_checksum profiles/r04_fetch_cal.json > /dev/null || exit 1
rm -rf $O/deflate_pmc && mv gpurun_out/prof $O/deflate_pmc
step configs
timeout -k 10 300 python3 tools/run_configs.py --config c5 > $O/c5.json 2> $O/c5.err || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c4 --scale 8 > $O/c4.json 2> $O/c4.err || exit 1
tail -n 3 $O/c5.json $O/c4.json
exit 0
