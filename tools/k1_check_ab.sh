# usage: bash tools/k1_check_ab.sh <tag> <variant> [rounds]: the K1 GPU parity tests on the product library, then
# tools/k1_ab.sh (product vs libnmz_gpu_<variant>.so)
tag=$1; v=$2; n=${3:-2}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -x -q --timeout 200 --timeout-method thread -k "k1 or wt or replayable" > gpurun_out/${tag}_k1_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/${tag}_k1_tests.log; exit $rc; }
tail -1 gpurun_out/${tag}_k1_tests.log
bash tools/k1_ab.sh $tag $v $n
