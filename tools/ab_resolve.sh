set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for v in base wake wake4; do
  if [ $v = base ]; then L=$PWD/sd-zlib_amd/lib/libsdz.so; else L=$PWD/sd-zlib_amd/lib/libsdz_$v.so; fi
  SDZ_LIB=$L timeout -k 10 200 python3 tools/run_c2.py --mode inflate --steps 3 > gpurun_out/ab_$v.log 2>&1 || exit 1
  SDZ_LIB=$L timeout -k 10 200 python3 tools/run_c2.py --mode distinct --steps 3 >> gpurun_out/ab_$v.log 2>&1 || exit 1
done
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_wake.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/ab_pt.log 2>&1
tail -2 gpurun_out/ab_pt.log
