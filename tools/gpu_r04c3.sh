# round-4 c3: K1 tests incl. prepared seed sets, end-to-end runs (stream over one seed set), timeline
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -x -q --timeout 200 --timeout-method thread -k "replayable or wt or k1 or plan or topk or seed" > gpurun_out/r04c3_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04c3_tests.log; exit $rc; }
tail -1 gpurun_out/r04c3_tests.log
bash tools/e2e_ab.sh r04c3 2 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r04c3_e2e_trace -o run -- python3 bench.py --legs replayable --no-cpu-baseline --e2e-traces 17 --steps 20 > gpurun_out/r04c3_e2e_trace.log 2>&1 || { tail -20 gpurun_out/r04c3_e2e_trace.log; exit 1; }
python3 tools/e2e_timeline.py gpurun_out/r04c3_e2e_trace > gpurun_out/r04c3_timeline.txt
head -14 gpurun_out/r04c3_timeline.txt
