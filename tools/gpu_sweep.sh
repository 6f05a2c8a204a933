#!/bin/bash
# bench sweep over an environment knob: tools/gpu_sweep.sh VAR "v1 v2 ..." [pipelines]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
VAR=$1; VALS=$2; PIPES=${3:-"3"}
for v in $VALS; do for d in $PIPES; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu --pipeline $d > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -20 gpurun_out/sw.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));k=d['kernels'];print('$VAR=$v pipeline',$d,round(d['value']),d['ms_per_step'],d['roofline']['frac'],d['config']['latency_ms_single_batch'],{n:v['us'] for n,v in k.items()})"
done; done
