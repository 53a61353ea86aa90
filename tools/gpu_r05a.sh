#!/bin/bash
# Round-5 checkpoint on HEAD (GPU box, repo root): -m gpu suite, smoke, the driver's bench command, a rocprofv3
# kernel trace of that same command, and K1's stall counters (one --pmc pass per run). Each step has its own
# limit; a crash / abort / time limit ends the script. usage: tools/gpu_r05a.sh <tag> [skip-tests]
tag=${1:-r05a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -3 $O/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
fi
timeout -k 10 400 python bench.py --full-record $O/bench_full.json > $O/bench.out 2> $O/bench.err || exit $?
tail -c 600 $O/bench.out
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --full-record $O/bench_prof_full.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.out 2> $O/trace.log || exit $?
bash $R/tools/kstalls.sh $tag/k1stalls k_replayable_sweep_wt --gpus 1 --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --full-record "" > /dev/null || exit $?
cat $O/k1stalls/summary.txt
exit 0
