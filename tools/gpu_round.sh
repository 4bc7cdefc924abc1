#!/bin/bash
# One GPU call of the round (run through gpurun): the -m gpu suite, the default bench line,
# then (PMC=1) the deflate leg's rocprofv3 passes.  Each GPU step has its own time limit and
# the first failure ends the call.  Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TEST_LIMIT:-700} python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
      ${PYTEST_ARGS:-} > gpurun_out/pt.log 2>&1
  rc=$?; tail -5 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 ${BENCH_LIMIT:-500} python3 bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; cat gpurun_out/bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
fi
if [ "${PMC:-0}" = 1 ]; then
  rm -rf gpurun_out/prof
  MODE=${PMC_MODE:-deflate} STREAMS=65536 STEPS=${PMC_STEPS:-1} PASSES="${PASSES:-kt fetch write sq1 sq2}" \
      bash tools/profile_inflate.sh || exit 1
fi
exit 0
