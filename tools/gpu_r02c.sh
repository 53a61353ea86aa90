set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_visualize.py tests/test_ed_gpu.py -k "visual or unique or zk or search" -x -v --timeout 200 --timeout-method thread > gpurun_out/r02c_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r02c_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02c_smoke.log 2>&1
