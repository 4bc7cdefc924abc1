cd "${GRAFT_REPO_ROOT}"
timeout -k 10 500 python3 -m pytest tests -m gpu -x -q -k "deflate" > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
for lib in ${LIBS:-libsdz.so}; do
  echo "== $lib"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 120 python3 tools/run_c2.py --mode deflate --streams 16384 --steps 2 2>&1 | grep -i "step\|parity\|error" || exit 1
done
