#!/bin/bash
# schedule comparison
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for cfg in "split 3 -1" "split 3 0" "split 4 -1" "streams 3 0"; do set -- $cfg
  MCAQ_MORPH_PRIO=$3 timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --schedule $1 --pipeline $2 > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -20 gpurun_out/sw.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$1',$2,'prio $3',round(d['value']),d['ms_per_step'],d['config']['latency_ms_single_batch'],d['config']['host_enqueue_us_per_step'])"
done
