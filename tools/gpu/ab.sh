#!/bin/bash
# Interleaved A/B of the built library against variant libraries
# tools/probe/ab/$v.so: ROUNDS (default 3) x (base, variants...) default bench
# lines (200 steps) plus each variant's kernel-timing fields.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=$1; shift
mkdir -p $R/gpurun_out/$T
cd $R
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in base "$@"; do
    if [ $v = base ]; then cp /tmp/base.so $L; else cp tools/probe/ab/$v.so $L; fi
    timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 ${BENCH_ARGS:-} > gpurun_out/$T/b_${v}_$r.json 2> gpurun_out/$T/b_${v}_$r.err || { cp /tmp/base.so $L; tail -5 gpurun_out/$T/b_${v}_$r.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/$T/b_${v}_$r.json')); k=d['kernels']
print('$v $r', round(d['value']), round(d['ms_per_step']*1e3,1), d['path_roofline']['frac'], 'quant', k['quant']['us'], k['quant']['us_in_sequence'], 'stats', k['stats']['us'], 'morph', k['morph_finalize']['us'])"
  done
done
cp /tmp/base.so $L
