#!/bin/bash
# Pipeline depth sweep (bench --pipeline D) for the built library and variant
# libraries tools/probe/ab/$v.so.  Tag $1, depths in $DEPTHS, variants $2...
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
  for d in ${DEPTHS:-3 4 5}; do
    timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 --pipeline $d > gpurun_out/$T/b_${v}_p$d.json 2> gpurun_out/$T/b_${v}_p$d.err || { cp /tmp/base.so $L; tail -5 gpurun_out/$T/b_${v}_p$d.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/$T/b_${v}_p$d.json')); print('$v p$d', round(d['value']), round(d['ms_per_step']*1e3,1), d['path_roofline']['frac'], d['config']['latency_ms_single_batch'])"
  done
done
cp /tmp/base.so $L
