#!/bin/bash
# HBM traffic per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE, separate passes,
# tools/pmc_summary.py) of the hook path (config 2, pipeline 1, eager) and
# the QAT step (config 5, eager), plus the rocprofv3 kernel stats / trace of
# the config-5 graph-replayed step.  Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r04_pmc}
mkdir -p $R/gpurun_out/$T
cd /tmp
for cfg in 2 5; do
  D=$R/gpurun_out/$T/config$cfg
  mkdir -p $D
  if [ $cfg = 2 ]; then A="--steps 8 --warmup 2 --pipeline 1 --eager --no-cpu --no-e2e"; else A="--config 5 --steps 4 --warmup 2 --eager --no-cpu"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d $D/pmc_$c -o run --output-format csv -- python3 $R/bench.py $A > $D/pmc_$c.log 2>&1 || { tail -5 $D/pmc_$c.log; exit 1; }
  done
  python3 $R/tools/pmc_summary.py $D > $D/pmc_summary.json || exit 1
  python3 -c "
import json; d=json.load(open('$D/pmc_summary.json'))
for k, v in d['kernels'].items():
    if k.startswith('mcaq'): print('  %-34s read %8.2f MB write %7.2f MB (%d launches)' % (k, v['read']/1e6, v['write']/1e6, v['launches']))"
done
D=$R/gpurun_out/$T/config5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu --steps 25 > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
f=$(find $D/prof -name "*kernel_stats.csv" | head -1); cp $f $D/kernel_stats_config5.csv
f=$(find $D/prof -name "*kernel_trace.csv" | head -1); cp $f $D/kernel_trace_config5.csv
python3 $R/tools/qat_timeline.py $D/kernel_trace_config5.csv > $D/timeline.txt; head -3 $D/timeline.txt; tail -1 $D/timeline.txt
