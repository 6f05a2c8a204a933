#!/bin/bash
# Round profile refresh: bench line, rocprofv3 kernel stats (default command and
# --pipeline 1), PMC traffic passes.  Tag = $1 (e.g. r01_v6).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r01_vX}
mkdir -p $R/gpurun_out/prof_$T
cd $R
timeout -k 10 300 python bench.py > gpurun_out/prof_$T/bench.json 2> gpurun_out/prof_$T/bench.err || { tail -20 gpurun_out/prof_$T/bench.err; exit 1; }
cat gpurun_out/prof_$T/bench.json
cd /tmp
for d in 3 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T/p$d -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu --pipeline $d > $R/gpurun_out/prof_$T/p$d.log 2>&1 || { tail -5 $R/gpurun_out/prof_$T/p$d.log; exit 1; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 --pipeline 1 --eager --no-cpu > $R/gpurun_out/pmc_$c.log 2>&1 || { tail -5 $R/gpurun_out/pmc_$c.log; exit 1; }
done
cd $R && python tools/pmc_summary.py gpurun_out > gpurun_out/prof_$T/pmc_summary.json && cat gpurun_out/prof_$T/pmc_summary.json
