#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per launch (separate passes) for the built library
# and variant libraries tools/probe/ab/$v.so, plus rocprofv3 --stats of a
# pipeline-1 bench for each.  Tag $1, variants $2...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=$1; shift
mkdir -p $R/gpurun_out/$T
L=$R/mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
for v in base "$@"; do
  if [ $v = base ]; then cp /tmp/base.so $L; else cp $R/tools/probe/ab/$v.so $L; fi
  D=$R/gpurun_out/$T/$v
  mkdir -p $D
  cd /tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $D/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 --pipeline 1 --eager --no-cpu --no-e2e > $D/pmc_$c.log 2>&1 || { cp /tmp/base.so $L; tail -5 $D/pmc_$c.log; exit 1; }
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_p1 -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --pipeline 1 --steps 200 > $D/prof_p1.log 2>&1 || { cp /tmp/base.so $L; tail -5 $D/prof_p1.log; exit 1; }
  cd $R
  f=$(find $D/prof_p1 -name "*kernel_stats.csv" | head -1); cp $f $D/kernel_stats_p1.csv
  python tools/pmc_summary.py $D > $D/pmc_summary.json
  echo "== $v"; python -c "
import json; d=json.load(open('$D/pmc_summary.json'))
for k, v in d['kernels'].items():
    if k.startswith('mcaq'): print('  %-28s read %8.2f MB write %7.2f MB (%d launches)' % (k, v['read']/1e6, v['write']/1e6, v['launches']))
print('  step', d['step_total']/1e6, 'MB')"
  cut -d, -f1-4 $D/kernel_stats_p1.csv | head -6
done
cp /tmp/base.so $L
