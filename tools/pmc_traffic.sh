#!/bin/bash
# HBM traffic per kernel launch from rocprofv3 PMC counters, one counter per pass
# (MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE cannot share a pass;
# FETCH_SIZE counts half the bytes of 16-byte streaming reads -> doubled by
# tools/pmc_summary.py).  Output: gpurun_out/pmc_<counter>/...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 2 --pipeline 1 --eager --no-cpu --no-e2e > $R/gpurun_out/pmc_$c.log 2>&1 || { tail -5 $R/gpurun_out/pmc_$c.log; exit 1; }
done
NB=$(python3 -c "import sys; sys.path.insert(0, '$R'); import bench; print(bench.LAUNCH_BATCHES)" 2>/dev/null || echo 1)
cd $R && MCAQ_PMC_BATCHES=$NB python tools/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.json && cat gpurun_out/pmc_summary.json
