#!/bin/bash
# Interleaved A/B of pass B per image vs batch-wide (bench --pass-b), streams
# and prefetch schedules, 3 rounds.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r04_passb}
mkdir -p $R/gpurun_out/$T
cd $R
for r in 1 2 3; do
  for v in image batch; do
    for s in streams; do
      timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 --pass-b $v --schedule $s > gpurun_out/$T/b_${v}_${s}_$r.json 2> gpurun_out/$T/b_${v}_${s}_$r.err || { tail -5 gpurun_out/$T/b_${v}_${s}_$r.err; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/$T/b_${v}_${s}_$r.json')); print('$v $s $r', round(d['value']), round(d['ms_per_step']*1e3,1), d['path_roofline']['frac'])"
    done
  done
done
