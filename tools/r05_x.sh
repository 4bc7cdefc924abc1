#!/bin/bash
# Round 5: the segment parse's size for small batches (down to 2^7): deflate parity, perf cases.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py tests/test_gpu_multi.py \
    -k "deflate or Deflate or dict or multi" > $O/x_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/x_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/x_dfl.log; exit $rc; }
timeout -k 10 60 python3 tools/lat/lat_big.py || exit 1
