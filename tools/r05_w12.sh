#!/bin/bash
# Round 5: on top of the 8-byte first compare -- a 12-byte one (PM_W12) and the refill threshold
# (PM_REFILL 12 / 16): C3 kernel time per build, alternated with the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05d
for v in ${VARIANTS:-default w12 rf12 rf16 default w12 rf12 rf16}; do
  lib=libsdz.so; [ $v != default ] && lib=libsdz_$v.so
  echo "== $v"
  SDZ_LIB=$PWD/sd-zlib_amd/lib/$lib timeout -k 10 200 python3 tools/run_c2.py --mode deflate --steps 3 | tail -1 || exit 1
done
