#!/bin/bash
# Round 5: k_dfl_match work-distribution knobs (PM_REFILL idle lanes per refill, PM_CHUNK
# positions per wave claim): C3 deflate kernel time per build, alternated with the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05d
for v in ${VARIANTS:-default rf12 rf16 rf24 ch256 default rf16}; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -2 || exit 1
done
