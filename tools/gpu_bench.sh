#!/bin/bash
# Bench variants + rocprof kernel stats of the default bench command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for d in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu --pipeline $d > gpurun_out/bench_p$d.json 2> gpurun_out/bench_p$d.err || { tail -20 gpurun_out/bench_p$d.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_p$d.json'));print('pipeline',$d,d['value'],d['ms_per_step'],d['roofline']['frac'],d['config']['latency_ms_single_batch'],d['kernels'])"
done
