#!/bin/bash
# in-kernel phase clocks of the deflate parse kernel (development aid; timing build of libsdz)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
SDZ_LIB=$PWD/sd-zlib_amd/lib/libsdz_timing.so SDZ_PHASE_TIMING=1 timeout -k 10 120 \
    python3 tools/run_c2.py --mode deflate --streams ${STREAMS:-65536} --steps 1 > gpurun_out/phase.log 2>&1
rc=$?; cat gpurun_out/phase.log; exit $rc
