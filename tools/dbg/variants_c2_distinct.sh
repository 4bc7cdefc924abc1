set -u
for v in ${VARIANTS:-libsdz.so}; do
  echo "== $v"
  SDZ_LIB=sd-zlib_amd/lib/$v timeout -k 10 120 python3 tools/run_c2.py --mode inflate --steps 3 2>&1 | grep "step 2" || exit 1
  SDZ_LIB=sd-zlib_amd/lib/$v timeout -k 10 120 python3 tools/run_c2.py --mode distinct --steps 3 2>&1 | grep "distinct" || exit 1
done
