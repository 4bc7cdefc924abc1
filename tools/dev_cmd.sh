# development GPU call: deflate parity (record path, 4-byte chain search), then C3 kernel splits
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py -x -q --timeout 200 --timeout-method thread -k "deflate" > gpurun_out/pt_dev.log 2>&1; rc=$?; tail -2 gpurun_out/pt_dev.log; [ $rc -ne 0 ] && exit $rc
for cfg in "SDZ_MATCH4=1"; do
  rm -rf gpurun_out/devkt
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/devkt -o run -- python3 tools/run_c2.py --mode deflate --steps 1 > gpurun_out/dev.log 2>&1 || exit 1
  echo "== $cfg"; grep "step" gpurun_out/dev.log; python3 tools/kt_db.py gpurun_out/devkt/run_results.db | head -3
  env $cfg SDZ_PHASE_TIMING=1 timeout -k 10 100 python3 tools/run_c2.py --mode deflate --steps 1 2>&1 | grep phases
done
