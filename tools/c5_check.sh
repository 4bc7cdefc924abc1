cd "${GRAFT_REPO_ROOT}"
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/run_configs.py --config c5 > gpurun_out/c5b.json 2>/dev/null || exit 1
timeout -k 10 120 python3 tools/run_c2.py --mode inflate --steps 2 2>&1 | grep step
