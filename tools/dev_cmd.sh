# development GPU call: the full GPU suite, then the bench line
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bench.json').read()); print(d['value'], d['roofline']['kernels_ms'], d['inflate_distinct']['roofline']['kernels_ms'], d['deflate']['kernel_ms'])"
