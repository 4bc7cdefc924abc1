# development GPU call: deflate with and without the 4-byte chain search by slice size and level
export TMPDIR=/tmp; mkdir -p gpurun_out
for m in 0 1; do
  echo "== SDZ_MATCH4=$m"
  for sl in 16384 32768 49152 131072; do for lv in 6 9; do
    n=$((65536 * 65536 / sl))
    SDZ_MATCH4=$m timeout -k 10 120 python3 tools/run_c2.py --mode deflate --steps 1 --level $lv --slice $sl --streams $n 2>&1 | grep step | sed "s/^/slice $sl L$lv /" || exit 1
  done; done
done
