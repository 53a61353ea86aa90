#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: 2 ranks on device 0, gloo for the collectives (RCCL refuses two
# ranks per device). Smaller configs[2]/[3] sizes keep it short. usage: tools/rehearse_n2.sh <tag>
TAG=${1:-n2}
mkdir -p gpurun_out
NMZ_BENCH_BACKEND=gloo NMZ_BENCH_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 \
  --ed-traces 20000 --random-total 2000000 --vis-traces 20000 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
