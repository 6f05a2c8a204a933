#!/bin/bash
# kernel trace of the pipelined bench (schedule given as $1, default streams)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/trace
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o run --output-format csv -- python3 $R/bench.py --steps 60 --warmup 5 --no-cpu --schedule ${1:-streams} > $R/gpurun_out/trace.log 2>&1 || { tail -5 $R/gpurun_out/trace.log; exit 1; }
tail -1 $R/gpurun_out/trace.log
