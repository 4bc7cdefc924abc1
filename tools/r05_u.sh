#!/bin/bash
# Round 5: one-buffer deflate: per-stream workgroup scan of the segment counts (k_lz_scan) and
# match segments sized to fill the chip (pm_seg): deflate parity (with the default policy and
# SDZ_PM_SEG=16384 forced), C3, the perf-case timings and trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
O=gpurun_out/r05
T="python3 -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py \
    -k "deflate or Deflate or dict" > $O/u_dfl.log 2>&1
rc=$?; echo "deflate parity rc=$rc: $(tail -1 $O/u_dfl.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/u_dfl.log; exit $rc; }
SDZ_PM_SEG=4096 timeout -k 10 600 $T tests/test_gpu_parity.py -k "deflate" > $O/u_dfl4k.log 2>&1
rc=$?; echo "deflate parity pm_seg 4096 rc=$rc: $(tail -1 $O/u_dfl4k.log)"; [ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" $O/u_dfl4k.log; exit $rc; }
timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
timeout -k 10 60 python3 tools/lat/lat_one.py || exit 1
for sg in 16384 8192 4096 2048; do echo "== pm_seg $sg"; SDZ_PM_SEG=$sg timeout -k 10 60 python3 tools/lat/lat_big.py | tail -1 || exit 1; done
bash tools/lat/lat_big_trace.sh
