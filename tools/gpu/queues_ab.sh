#!/bin/bash
# Pipeline depth x HW queue count sweep for the built library and variants.
# Tag $1, variants $2...; depths $DEPTHS, queue counts $QUEUES.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=$1; shift
mkdir -p $R/gpurun_out/$T
cd $R
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
for v in base "$@"; do
  if [ $v = base ]; then cp /tmp/base.so $L; else cp tools/probe/ab/$v.so $L; fi
  for q in ${QUEUES:-4 8}; do
    for d in ${DEPTHS:-3 4 6}; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 --pipeline $d > gpurun_out/$T/b_${v}_q${q}_p$d.json 2> gpurun_out/$T/b_${v}_q${q}_p$d.err || { cp /tmp/base.so $L; tail -5 gpurun_out/$T/b_${v}_q${q}_p$d.err; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/$T/b_${v}_q${q}_p$d.json')); print('$v q$q p$d', round(d['value']), round(d['ms_per_step']*1e3,1), d['path_roofline']['frac'])"
    done
  done
done
cp /tmp/base.so $L
