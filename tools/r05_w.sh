#!/bin/bash
# Round 5: one-buffer deflate with shorter parse segments (SDZ_LZ_SHIFT 9 -> 6) and the
# chain units as they are: the perf-case timings for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
for sh in 9 8 7 6; do echo "== lz_shift $sh"; SDZ_LZ_SHIFT=$sh timeout -k 10 60 python3 tools/lat/lat_big.py | tail -2 || exit 1; done
