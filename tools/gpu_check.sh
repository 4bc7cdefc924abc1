#!/bin/bash
# GPU round trip used during development (run through gpurun): parity tests, then
# C2 inflate timing.  Each GPU step has its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${TEST_LIMIT:-400} python3 -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 ${C2_LIMIT:-180} python3 tools/run_c2.py --mode inflate --streams ${STREAMS:-65536} --steps ${STEPS:-3} > gpurun_out/c2.log 2>&1
rc=$?; cat gpurun_out/c2.log | tail -5; exit $rc
