# round-4 development GPU call: the wave decoder (SDZ_WDEC=1: tokens for k_inflate_resolve) against
# the inflate parity tests, then phase clocks and C2 / distinct timings against the lane decoder
export TMPDIR=/tmp; mkdir -p gpurun_out
K="${K:-inflate or fixtures or c2 or corrupted or chunkwise or dictionary or stored or trailing or need_bits or small_rounds or output_slot or concurrent or checksums or api_mirror or repetitive}"
SDZ_WDEC=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/r04_pt1.log 2>&1; rc=$?
echo "wdec tests rc=$rc: $(tail -1 gpurun_out/r04_pt1.log)"
[ $rc -eq 0 ] || { grep -m8 -E "Error|assert|FAIL" gpurun_out/r04_pt1.log; exit $rc; }
PMODES=1 WMODES="${WMODES:-0 1}" bash tools/wdec_phase.sh
