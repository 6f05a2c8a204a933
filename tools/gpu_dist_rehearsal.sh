#!/bin/bash
# Functional rehearsal of bench.py's N>1 path on one GPU: 2 ranks, gloo backend
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
MCAQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 12 --warmup 3 --no-cpu > gpurun_out/dist.json 2> gpurun_out/dist.err || { tail -30 gpurun_out/dist.err; exit 1; }
cat gpurun_out/dist.json
