# usage: bash tools/gpu_quick.sh <tag> <pytest selection args...>
# Runs the selected GPU tests, then smoke() unless a test run ended abnormally (not a plain test failure).
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest "$@" -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${tag}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
