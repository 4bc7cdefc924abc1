# development GPU call: deflate parity with the LDS tail search, then C3 and C5 kernel splits
export TMPDIR=/tmp; mkdir -p gpurun_out
for t in 0 1; do
  SDZ_TAIL_LDS=$t timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py -x -q --timeout 240 --timeout-method thread -k "deflate or dict" > gpurun_out/pt_dev$t.log 2>&1; rc=$?; tail -1 gpurun_out/pt_dev$t.log; [ $rc -ne 0 ] && exit $rc
done
rm -rf gpurun_out/devkt
SDZ_TAIL_LDS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/devkt -o run -- python3 tools/run_c2.py --mode deflate --steps 1 > gpurun_out/dev.log 2>&1 || exit 1
grep "step" gpurun_out/dev.log; python3 tools/kt_db.py gpurun_out/devkt/run_results.db | grep tail
rm -rf gpurun_out/devkt
SDZ_TAIL_LDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/devkt -o run -- python3 tools/run_configs.py --config c5 > gpurun_out/dev5.log 2>&1 || exit 1
grep -o '"deflate_kernel_ms": [0-9.]*\|"parity": [a-z]*' gpurun_out/dev5.log; python3 tools/kt_db.py gpurun_out/devkt/run_results.db | grep tail
