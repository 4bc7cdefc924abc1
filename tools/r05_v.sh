#!/bin/bash
# Round 5: k_dfl_encode on 1,024 threads for few streams (k_dfl_encode_t<1024>): deflate parity,
# the perf-case timings, C3 (the 256-thread path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py \
    -k "deflate or Deflate or dict" > $O/v_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/v_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/v_dfl.log; exit $rc; }
timeout -k 10 60 python3 tools/lat/lat_big.py || exit 1
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
