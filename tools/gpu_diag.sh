#!/bin/bash
# diagnostics: morph stage stamps, per-scale pass times, kernel trace of the pipelined bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python tools/prof_morph_stamps.py 2 > gpurun_out/stamps.log 2>&1; cat gpurun_out/stamps.log | grep -v amdgpu.ids
cd tools && timeout -k 10 120 python prof_stats.py 2 > ../gpurun_out/pstats.log 2>&1; grep -v amdgpu.ids ../gpurun_out/pstats.log; cd ..
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --no-cpu --no-e2e > $R/gpurun_out/trace.log 2>&1 || { tail -5 $R/gpurun_out/trace.log; exit 1; }
cd $R && python tools/trace_analyze.py $(ls gpurun_out/trace/*/run_kernel_trace.csv gpurun_out/trace/run_kernel_trace.csv 2>/dev/null | head -1) 200
