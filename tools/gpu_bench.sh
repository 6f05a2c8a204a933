#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for ex in 0 1; do for d in 2 3; do
  MCAQ_MORPH_EXCLUSIVE=$ex timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu --pipeline $d > gpurun_out/bench_p$d.json 2> gpurun_out/bench_p$d.err || { tail -20 gpurun_out/bench_p$d.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_p$d.json'));k=d['kernels'];print('excl',$ex,'pipeline',$d,d['value'],d['ms_per_step'],d['roofline']['frac'],d['config']['latency_ms_single_batch'],k['stats']['us'],k['morph_finalize']['us'],k['quant']['us'])"
done; done
