#!/bin/bash
# the whole GPU suite (as the driver runs it) and smoke(), then the facade and Node latencies
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/full_gpu.log 2>&1; rc=$?
echo "gpu suite rc=$rc: $(tail -1 gpurun_out/full_gpu.log)"
[ $rc -eq 0 ] || { grep -m12 -E "Error|assert|FAIL|failed" gpurun_out/full_gpu.log; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 || exit 1
[ -n "${LAT:-1}" ] && timeout -k 10 300 python3 tools/facade_prof.py 2>&1 | tail -8
[ -n "${NODE:-1}" ] && which node > /dev/null && timeout -k 10 300 node tests/node/perf.mjs 2>&1 | tail -3
[ -n "${C3:-}" ] && timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 2 2>&1 | tail -2
exit 0
