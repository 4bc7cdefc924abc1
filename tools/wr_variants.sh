cd ${GRAFT_REPO_ROOT}
export TMPDIR=/tmp
for l in ${LIBS:-libsdz.so}; do
  echo "== $l"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$l timeout -k 10 120 python3 tools/run_c2.py --mode inflate --streams 65536 --steps 2 | tail -1 || exit 1
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$l timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/w_$l -o run --output-format csv -- python3 tools/run_c2.py --mode inflate --streams 65536 --steps 1 > /dev/null 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/w_$l | grep -E "resolve.*WRITE"
done
