#!/bin/bash
# Round 5: in-kernel phase clocks (libsdz_timing.so, SDZ_PHASE_TIMING=1) of the inflate kernels on C2
# and on the distinct 64 KiB streams.  Resolve (first 8 streams' emitter waves): dbg[0] scan, [1] chain
# wait, [2] copy rounds, [4] finality wait cycles, [6] emit rounds, [7] idle polls; decode: [8] cold
# cycles, [9] hot cycles, [10] cold runs, [11] hot epochs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r05
for m in inflate distinct; do
  echo "== $m"
  SDZ_PHASE_TIMING=1 SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_timing.so timeout -k 10 200 python3 tools/run_c2.py --mode $m --steps 1 2>&1 | grep -E "phases|kernel" | tail -3 || exit 1
done
