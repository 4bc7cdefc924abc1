# development GPU call: parity of the 4-byte chain search, then its C3 kernel split
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k 4byte > gpurun_out/pt_dev.log 2>&1; rc=$?; tail -2 gpurun_out/pt_dev.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/devkt
SDZ_MATCH4=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/devkt -o run -- python3 tools/run_c2.py --mode deflate --steps 1 > gpurun_out/dev.log 2>&1 || exit 1
grep "step" gpurun_out/dev.log
