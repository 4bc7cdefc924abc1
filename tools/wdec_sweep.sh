#!/bin/bash
# wave vs lane path by batch size (paradiselost copies, and distinct 64 KiB streams): where the
# wave decoder stops paying (inflate_wave_policy's kWdAutoStreams)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out
for m in inflate distinct; do
  for n in 4096 8192 16384 32768; do
    for w in 1 0; do
      r=$(SDZ_WDEC=$w timeout -k 10 120 python3 tools/run_c2.py --mode $m --streams $n --steps 2 2>&1 | tail -1) || { echo "failed $m $n $w"; exit 1; }
      echo "$m streams $n SDZ_WDEC=$w: $r"
    done
  done
done
