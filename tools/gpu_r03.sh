#!/bin/bash
# usage (GPU box, repo root): bash tools/gpu_r03.sh <tag> "<pytest selection>" "<bench legs>" ["<bench legs 2>"]
# GPU tests first (their failures do not stop the bench; a crash, abort or time limit does), then one or two
# bench runs of the given legs. Every step has its own time limit.
tag=$1; sel=$2; legs=$3; legs2=$4
mkdir -p gpurun_out
if [ -n "$sel" ]; then
  timeout -k 10 700 python -u -m pytest $sel -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/${tag}_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$legs" ]; then
  timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --legs $legs > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
fi
if [ -n "$legs2" ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --legs $legs2 > gpurun_out/${tag}_bench2.json 2> gpurun_out/${tag}_bench2.err || exit $?
fi
exit 0
