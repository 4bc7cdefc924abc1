#!/bin/bash
# wave decoder phase clocks (SDZ_TIMING build; development aid): C2, distinct and one stream;
# then plain timings of the wave decoder modes (WMODES) against the lane decoder
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${PMODES:-1}; do
  for m in "inflate --streams 65536" "distinct --streams 65536" "inflate --streams 1"; do
    echo "== phases wdec=$w $m"
    SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_timing.so SDZ_PHASE_TIMING=1 SDZ_WDEC=$w timeout -k 10 200 \
        python3 tools/run_c2.py --mode $m --steps 1 2>&1 | grep -E "phases|kernel" || exit 1
  done
done
for w in ${WMODES:-1 2}; do
  for m in inflate distinct; do
    SDZ_WDEC=$w timeout -k 10 200 python3 tools/run_c2.py --mode $m --steps 2 2>&1 | tail -1 | sed "s/^/wdec=$w /" || exit 1
  done
done
