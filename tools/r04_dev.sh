# round-4 development GPU call: the wave decoder (SDZ_WDEC=1) against the inflate parity tests,
# then C2 / distinct timings with the lane decoder and the wave decoder
export TMPDIR=/tmp; mkdir -p gpurun_out
K="${K:-inflate or fixtures or c2 or corrupted or chunkwise or dictionary or stored or trailing or need_bits or small_rounds or output_slot or concurrent or checksums or api_mirror or repetitive}"
SDZ_WDEC=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/r04_pt.log 2>&1; rc=$?
tail -5 gpurun_out/r04_pt.log
[ $rc -eq 0 ] || exit $rc
for w in 0 1; do
  SDZ_WDEC=$w timeout -k 10 120 python3 tools/run_c2.py --mode inflate --steps 3 2>&1 | tail -1 | sed "s/^/wdec=$w C2 /"
  SDZ_WDEC=$w timeout -k 10 200 python3 tools/run_c2.py --mode distinct --steps 3 2>&1 | tail -1 | sed "s/^/wdec=$w distinct /"
done
