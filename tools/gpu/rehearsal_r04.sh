#!/bin/bash
# Functional rehearsal of the N = 2 paths on the one-GPU box (gloo, both ranks
# on cuda:0; never a measurement): config 2 hook path and config 5 QAT step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_rehearsal
for c in 2 5; do
  MCAQ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + c)) bench.py --gpus 2 --config $c --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/r04_rehearsal/gloo_n2_config$c.json 2> gpurun_out/r04_rehearsal/gloo_n2_config$c.err || { tail -20 gpurun_out/r04_rehearsal/gloo_n2_config$c.err; exit 1; }
  tail -c 600 gpurun_out/r04_rehearsal/gloo_n2_config$c.json; echo
done
