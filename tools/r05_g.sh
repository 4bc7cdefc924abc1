#!/bin/bash
# Round 5: the fault-narrowing runs of the hot_epoch-inlined variant (tools/r05_f.sh, HIP-reported
# faults only), then the round's measurement (tools/r05_measure.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r05_f.sh
bash tools/r05_measure.sh
