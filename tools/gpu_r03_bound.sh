#!/bin/bash
# r03: step bounds (streaming only / morph only) + kernel trace of the default bench
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_bound}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 200 python -u tools/probe/bound_probe.py > gpurun_out/$T/bound.txt 2>&1; rc=$?; cat gpurun_out/$T/bound.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/$T/trace -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 10 --no-cpu --no-e2e > $R/gpurun_out/$T/trace.log 2>&1 || { tail -5 $R/gpurun_out/$T/trace.log; exit 1; }
cd $R && f=$(ls gpurun_out/$T/trace/*/*kernel_trace.csv gpurun_out/$T/trace/*kernel_trace.csv 2>/dev/null | head -1) && python tools/trace_analyze.py $f 600 && tail -1 gpurun_out/$T/trace.log | cut -c1-200
