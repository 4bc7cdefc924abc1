# development GPU call: deflate parity, then the C3 kernel split
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py -x -q --timeout 200 --timeout-method thread -k "deflate or dict" > gpurun_out/pt_dev.log 2>&1; rc=$?; tail -1 gpurun_out/pt_dev.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/devkt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/devkt -o run -- python3 tools/run_c2.py --mode deflate --steps 1 > gpurun_out/dev.log 2>&1 || exit 1
grep "step" gpurun_out/dev.log; python3 tools/kt_db.py gpurun_out/devkt/run_results.db | head -8
