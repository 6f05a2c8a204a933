#!/bin/bash
# Quick GPU iteration: selected GPU tests ($2, pytest -k expression) then a
# 200-step default bench line and the rocprofv3 kernel stats of a pipeline-1
# and a pipeline-3 bench.  Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-quick}
K=${2:-parity}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$K" > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/$T/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 200 > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err || { tail -5 gpurun_out/$T/b.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/$T/b.json')); print('bench', d['value'], d['ms_per_step'], d['path_roofline']['frac'], d['config']['raw_window_ms_per_step'], d['kernels']['stats']['us'], d['kernels']['morph_finalize']['us'], d['kernels']['quant']['us'])"
cd /tmp
for p in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof_p$p -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --pipeline $p --steps 200 > $R/gpurun_out/$T/prof_p$p.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof_p$p.log; exit 1; }
  f=$(find $R/gpurun_out/$T/prof_p$p -name "*kernel_stats.csv" | head -1); cp $f $R/gpurun_out/$T/kernel_stats_p$p.csv
  cut -d, -f1-4 $R/gpurun_out/$T/kernel_stats_p$p.csv | head -8
done
