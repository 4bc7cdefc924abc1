#!/bin/bash
# Round 5: round drivers without memset launches (k_inflate_wcold / k_fz_merge zero the counters
# the next kernel fills) and with pinned read-back words: parity of the wave decoder and of the
# L1-L3 rounds, then the one-buffer perf-case timings and their trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 800 $T tests/test_gpu_wdec.py tests/test_gpu_parity.py tests/test_gpu_multi.py > $O/t_par.log 2>&1
rc=$?; echo "parity rc=$rc: $(tail -1 $O/t_par.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/t_par.log; exit $rc; }
bash tools/lat/lat_big_trace.sh
