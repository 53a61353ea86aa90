# usage: bash tools/gpu_bench.sh <tag> [pytest selection...]: optional GPU tests, then the default bench
tag=$1; shift
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/${tag}_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 500 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
