# round-4 development GPU call: the wave decoder (SDZ_WDEC=1: tokens for k_inflate_resolve;
# SDZ_WDEC=2: fused, the wave writes the bytes) against the inflate parity tests, then C2 /
# distinct timings for the lane decoder and both wave-decoder modes
export TMPDIR=/tmp; mkdir -p gpurun_out
K="${K:-inflate or fixtures or c2 or corrupted or chunkwise or dictionary or stored or trailing or need_bits or small_rounds or output_slot or concurrent or checksums or api_mirror or repetitive}"
for w in ${WMODES:-2 1}; do
  SDZ_WDEC=$w timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/r04_pt$w.log 2>&1; rc=$?
  echo "wdec=$w tests rc=$rc: $(tail -1 gpurun_out/r04_pt$w.log)"
  [ $rc -eq 0 ] || { grep -m5 -E "Error|assert|FAIL" gpurun_out/r04_pt$w.log; exit $rc; }
done
for w in 0 ${WMODES:-2 1}; do
  SDZ_WDEC=$w timeout -k 10 120 python3 tools/run_c2.py --mode inflate --steps 3 2>&1 | tail -1 | sed "s/^/wdec=$w C2 /"
  SDZ_WDEC=$w timeout -k 10 200 python3 tools/run_c2.py --mode distinct --steps 3 2>&1 | tail -1 | sed "s/^/wdec=$w distinct /"
done
