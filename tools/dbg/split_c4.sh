#!/bin/bash
# C4 at 1/8 share with and without the split path, plus its parity tests (through gpurun)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py -m gpu || exit 1
SDZ_SPLIT=0 timeout -k 10 300 python3 tools/run_configs.py --config c4 --scale 8 || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c4 --scale 8
