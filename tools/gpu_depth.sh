#!/bin/bash
# pipeline depth x HW queues sweep
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for q in 4 8; do for d in 3 4 6; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu --pipeline $d > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -20 gpurun_out/sw.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('queues',$q,'pipeline',$d,round(d['value']),d['ms_per_step'],d['config']['latency_ms_single_batch'])"
done; done
