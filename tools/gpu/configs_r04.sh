#!/bin/bash
# Round 4: bench lines + rocprofv3 kernel stats (pipeline 1) for configs 3
# and 4, and the QAT step (config 5) kernel stats.  Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r04_configs}
mkdir -p $R/gpurun_out/$T
cd $R
for c in 3 4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-e2e > gpurun_out/$T/bench_config$c.json 2> gpurun_out/$T/bench_config$c.err || { tail -8 gpurun_out/$T/bench_config$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/$T/bench_config$c.json')); print('config $c', round(d['value']), round(d['ms_per_step']*1e3,1), 'path', d['path_roofline']['frac'], 'pass2', d['roofline']['frac'], d['roofline']['us_per_launch'])"
done
cd /tmp
for c in 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof_c$c -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu --no-e2e --pipeline 1 --steps 100 > $R/gpurun_out/$T/prof_c$c.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof_c$c.log; exit 1; }
  f=$(find $R/gpurun_out/$T/prof_c$c -name "*kernel_stats.csv" | head -1); cp $f $R/gpurun_out/$T/kernel_stats_config${c}_p1.csv
  cut -d, -f1-4 $R/gpurun_out/$T/kernel_stats_config${c}_p1.csv | head -6
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof_c5 -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu --steps 25 > $R/gpurun_out/$T/prof_c5.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof_c5.log; exit 1; }
f=$(find $R/gpurun_out/$T/prof_c5 -name "*kernel_stats.csv" | head -1); cp $f $R/gpurun_out/$T/kernel_stats_config5.csv
f=$(find $R/gpurun_out/$T/prof_c5 -name "*kernel_trace.csv" | head -1); cp $f $R/gpurun_out/$T/kernel_trace_config5.csv
python3 $R/tools/qat_stats.py $R/gpurun_out/$T/kernel_stats_config5.csv 30
