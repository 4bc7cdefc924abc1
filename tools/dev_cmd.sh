# development GPU call: the full GPU suite and smoke()
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()"
