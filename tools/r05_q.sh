#!/bin/bash
# Round 5: the Node facade's inflate() on the one-shot path: node smoke (errors against the
# Inflater path), the Node perf case.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
timeout -k 10 300 node tests/node/smoke.mjs > gpurun_out/r05/q_smoke.log 2>&1
rc=$?; echo "node smoke rc=$rc"; grep -E "FAIL|inflate (truncated|bad)" gpurun_out/r05/q_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 node tests/node/perf.mjs 2>&1 | tail -2
