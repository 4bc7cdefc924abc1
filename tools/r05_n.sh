#!/bin/bash
# Round 5: small calls without markers between launches (kernel-time events only for multi-GPU
# stats; pool / staging done events deferred to after the copy back): the GPU suite's host-path
# tests, the multi-GPU tests, latency, the trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_gpu_dict.py tests/test_gpu_multi.py tests/test_gpu_stream.py \
    tests/test_gpu_deflate_stream.py > $O/n_par.log 2>&1
rc=$?; echo "parity rc=$rc: $(tail -1 $O/n_par.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/n_par.log; exit $rc; }
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
bash tools/lat/lat_trace.sh
