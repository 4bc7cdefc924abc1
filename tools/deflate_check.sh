#!/bin/bash
# deflate parity tests, then a kernel-trace profile of C3 (64 Ki x 64 KiB, L6) -- development aid
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
R=$PWD
timeout -k 10 ${TEST_LIMIT:-500} python3 -m pytest tests -m gpu -x -q -k "${PYK:-deflate or api or smoke}" > gpurun_out/pt.log 2>&1
rc=$?; tail -15 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dk -o run --output-format csv -- \
    python3 $R/tools/run_c2.py --mode deflate --streams ${STREAMS:-65536} --steps 1 > $R/gpurun_out/dk.log 2>&1
rc=$?; grep -v "^[WIE]20" $R/gpurun_out/dk.log | tail -3
f=$(ls $R/gpurun_out/dk/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -14
exit $rc
