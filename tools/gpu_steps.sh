#!/bin/bash
# One GPU call as a list of named steps (run through gpurun), e.g.
#   gpurun -- 'bash tools/gpu_steps.sh OUT=r06a "t:tests/test_gpu_lane.py" c2 "c2:SDZ_RESOLVE=0" dist'
# Steps (each under its own time limit; the first failure ends the call):
#   t:[ENV=V,...|]<pytest args>  pytest -m gpu on the given files / -k expression (with that environment)
#   suite               the whole -m gpu suite
#   c2[:ENV=V,...]      tools/run_c2.py --mode inflate (C2), with the given environment
#   dist[:ENV=V,...]    tools/run_c2.py --mode distinct (64 Ki distinct 64 KiB streams)
#   mixed[:ENV=V,...]   tools/run_c2.py --mode mixed (the bench's C4-shaped leg, one rank)
#   c3[:ENV=V,...]      tools/run_c2.py --mode deflate (C3)
#   bench[:ARGS]        bench.py with the given arguments (commas become spaces)
#   kt:<mode>[:ENV=V,...]  rocprofv3 kernel trace + stats of run_c2.py --mode <mode> (into kt_<mode>_<step>)
#   pmc:<mode>:<set>    rocprofv3 --pmc pass <set> (sq1 sq2 sq3 fetch write) of run_c2.py --mode <mode>
#   ktbench[:ARGS]      rocprofv3 kernel trace + stats of bench.py with the given arguments (into kt_bench_<step>)
#   smoke               __graft_entry__.smoke()
#   configs             tools/run_configs.py (C4 / C5)
#   node                tests/node/smoke.mjs (the drop-in facade)
# Outputs under gpurun_out/$OUT/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=r06
if [[ "${1:-}" == OUT=* ]]; then OUT=${1#OUT=}; shift; fi
O=gpurun_out/$OUT
mkdir -p $O
n=0
envrun() {  # "A=1,B=2" cmd... -> runs cmd with that environment
    local e=$1; shift
    if [ -n "$e" ]; then env ${e//,/ } "$@"; else "$@"; fi
}
declare -A PMC=(
  [sq1]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
  [sq2]="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
  [sq3]="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
  [fetch]="FETCH_SIZE"
  [write]="WRITE_SIZE"
)
for st in "$@"; do
  n=$((n + 1))
  name=${st%%:*}; arg=""; [[ "$st" == *:* ]] && arg=${st#*:}
  log=$O/$(printf %02d $n)_$name.log
  echo "== step $n: $st" | tee -a $O/steps.txt
  case $name in
    t) e=""; a=$arg; [[ "$arg" == *"|"* ]] && { e=${arg%%|*}; a=${arg#*|}; }
       envrun "$e" timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread $a > $log 2>&1 ;;
    suite) timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $log 2>&1 ;;
    c2) envrun "$arg" timeout -k 10 300 python3 tools/run_c2.py --mode inflate --steps 3 > $log 2>&1 ;;
    dist) envrun "$arg" timeout -k 10 300 python3 tools/run_c2.py --mode distinct --steps 3 > $log 2>&1 ;;
    c3) envrun "$arg" timeout -k 10 300 python3 tools/run_c2.py --mode deflate --steps 3 > $log 2>&1 ;;
    mixed) envrun "$arg" timeout -k 10 300 python3 tools/run_c2.py --mode mixed --steps 2 > $log 2>&1 ;;
    node) timeout -k 10 300 node tests/node/smoke.mjs > $log 2>&1 ;;
    bench) timeout -k 10 600 python3 bench.py ${arg//,/ } > $log 2> $log.err ;;
    kt) mode=${arg%%:*}; e=""; [[ "$arg" == *:* ]] && e=${arg#*:}
        d=$O/kt_${mode}_$n; rm -rf $d
        envrun "$e" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
            python3 tools/run_c2.py --mode $mode --steps 2 > $log 2>&1 ;;
    pmc) mode=${arg%%:*}; set_=${arg#*:}
         rm -rf $O/pmc_${mode}_$set_
         timeout -s KILL 240 rocprofv3 --pmc ${PMC[$set_]} -d $O/pmc_${mode}_$set_ -o run --output-format csv -- \
            python3 tools/run_c2.py --mode $mode --steps 1 > $log 2>&1 ;;
    ktbench) d=$O/kt_bench_$n; rm -rf $d
        timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
            python3 bench.py ${arg//,/ } > $log 2> $log.err ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $log 2>&1 ;;
    configs) timeout -k 10 600 python3 tools/run_configs.py $arg > $log 2>&1 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
  rc=$?
  tail -4 $log | tee -a $O/steps.txt
  echo "rc=$rc" | tee -a $O/steps.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
