#!/bin/bash
# Full GPU check on HEAD (GPU box, repo root): -m gpu suite, smoke, default bench; each step under its own limit,
# a crash / abort / time limit ends the script. usage: tools/gpu_full.sh <tag>
tag=${1:-full}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${tag}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
exit 0
