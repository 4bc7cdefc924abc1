# development GPU call: the full GPU suite, C3 walk counters of k_dfl_match, the C5 config
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
SDZ_PHASE_TIMING=1 timeout -k 10 100 python3 tools/run_c2.py --mode deflate --steps 1 2>&1 | grep "phases\|step" || exit 1
timeout -k 10 300 python3 tools/run_configs.py --config c5 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
cat gpurun_out/c5.json
