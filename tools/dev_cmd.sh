# development GPU call: deflate parity, then C3 kernel splits of library variants
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py -x -q --timeout 200 --timeout-method thread -k "deflate" > gpurun_out/pt_dev.log 2>&1; rc=$?; tail -2 gpurun_out/pt_dev.log; [ $rc -ne 0 ] && exit $rc
for v in "" pw2 pw2r4; do
  lib=$PWD/sd-zlib_amd/lib/libsdz.so; [ -n "$v" ] && lib=$PWD/sd-zlib_amd/lib/libsdz_$v.so
  rm -rf gpurun_out/devkt
  SDZ_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/devkt -o run -- python3 tools/run_c2.py --mode deflate --steps 1 > gpurun_out/dev.log 2>&1 || exit 1
  echo "== ${v:-default}"; grep "step" gpurun_out/dev.log; python3 tools/kt_db.py gpurun_out/devkt/run_results.db | head -1
done
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_pw2.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "deflate_record or 4byte or deflate_all" > gpurun_out/pt_dev2.log 2>&1; rc=$?; tail -1 gpurun_out/pt_dev2.log; exit $rc
