# development GPU call: C3 with the segment-parallel parse at forced segment sizes
export TMPDIR=/tmp; mkdir -p gpurun_out
for sh in 16 15 14 13; do
  rm -rf gpurun_out/devkt
  SDZ_LZ_SHIFT=$sh timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/devkt -o run -- python3 tools/run_c2.py --mode deflate --steps 1 > gpurun_out/dev.log 2>&1 || exit 1
  echo "== shift $sh"; grep "step" gpurun_out/dev.log; python3 tools/kt_db.py gpurun_out/devkt/run_results.db | grep "k_lz\|k_dfl_parse"
done
