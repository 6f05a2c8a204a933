#!/bin/bash
# The driver's default bench command (CPU baseline and end-to-end leg
# included), then rocprofv3 kernel stats of the default bench at pipeline 1
# and pipeline 3.  Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r04_prof}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 400 python bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || { tail -5 gpurun_out/$T/bench_default.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/$T/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['path_roofline']['frac'], d['roofline']['frac'], d['cpu_baseline']['value'])"
cd /tmp
for p in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof_p$p -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --pipeline $p --steps 200 > $R/gpurun_out/$T/prof_p$p.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof_p$p.log; exit 1; }
  f=$(find $R/gpurun_out/$T/prof_p$p -name "*kernel_stats.csv" | head -1); cp $f $R/gpurun_out/$T/kernel_stats_p$p.csv
  cut -d, -f1-4 $R/gpurun_out/$T/kernel_stats_p$p.csv | head -8
done
