#!/bin/bash
# One GPU call made of named steps (round 6: replaces the one-shot scripts of scripts/runs/, indexed in
# scripts/runs/INDEX.md). Every step runs under its own time limit and writes under gpurun_out/<tag>/; the first
# step that fails ends the call (a GPU step that faults, aborts or times out must not be followed by another).
# Usage (from the repo root, via gpurun): scripts/gpu_run.sh <tag> <step> [<step> ...]
#   tests[=<pytest args>]        the -m gpu suite (or the given selection), -x, thread timeouts
#   smoke                        __graft_entry__.smoke()
#   bench[=<bench.py args>]      one bench line -> bench_<n>.json
#   probe=<script> [args]        python3 scripts/<script> args -> probe_<n>.txt
#   pmc[=<bench.py args>]        the PMC passes of scripts/prof_pmc.sh + their summary (pmc_summary.txt)
#   rocprof[=<bench.py args>]    rocprofv3 --kernel-trace --stats of one bench run -> stats/
set -o pipefail
TAG=$1; shift
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  echo "== step $n: $step" | tee -a $OUT/steps.log
  case $name in
    tests)
      sel=${arg:-"tests -m gpu"}
      timeout -k 10 600 python -u -m pytest $sel -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$n.txt 2>&1
      rc=$?; tail -4 $OUT/pytest_$n.txt ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$n.txt 2>&1
      rc=$?; tail -2 $OUT/smoke_$n.txt ;;
    bench)
      timeout -k 10 400 python -u bench.py $arg > $OUT/bench_$n.json 2> $OUT/bench_$n.err
      rc=$?; tail -1 $OUT/bench_$n.json; [ $rc -ne 0 ] && tail -20 $OUT/bench_$n.err ;;
    probe)
      timeout -k 10 400 python3 -u scripts/$arg > $OUT/probe_$n.txt 2>&1
      rc=$?; tail -30 $OUT/probe_$n.txt ;;
    pmc)
      scripts/prof_pmc.sh $TAG/pmc $arg && \
        python3 scripts/pmc_summary.py --json $OUT/pmc_traffic.json --config "1920x1080 K=0.25 moving" $OUT/pmc/*/ \
          > $OUT/pmc_summary.txt
      rc=$?; head -30 $OUT/pmc_summary.txt ;;
    rocprof)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
        python3 $R/bench.py $arg > $OUT/stats.log 2>&1)
      rc=$?; cat $(find $OUT/stats -name "*kernel_stats.csv") 2>/dev/null | head -12 ;;
    *)
      echo "unknown step $name"; rc=2 ;;
  esac
  if [ $rc -ne 0 ]; then echo "step $n ($name) ended with $rc: stopping" | tee -a $OUT/steps.log; exit $rc; fi
done
