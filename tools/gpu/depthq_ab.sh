#!/bin/bash
# Pipeline depth x hardware queues (GPU_MAX_HW_QUEUES) for the built library,
# two interleaved rounds.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-depthq}
mkdir -p $R/gpurun_out/$T
cd $R
for r in 1 2; do
  for qd in "4 3" "8 3" "8 4" "8 5" "8 6" "16 4" "16 6"; do
    set -- $qd; q=$1; d=$2
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 --pipeline $d > gpurun_out/$T/b_q${q}_p${d}_$r.json 2> gpurun_out/$T/b_q${q}_p${d}_$r.err || { tail -5 gpurun_out/$T/b_q${q}_p${d}_$r.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/$T/b_q${q}_p${d}_$r.json')); print('q$q p$d r$r', round(d['value']), round(d['ms_per_step']*1e3,1), d['path_roofline']['frac'])"
  done
done
