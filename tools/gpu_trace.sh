#!/bin/bash
# parity tests, stats diagnostics, and a kernel trace of the pipelined bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
cd tools && timeout -k 10 120 python prof_stats.py 2 > ../gpurun_out/pstats.log 2>&1; cat ../gpurun_out/pstats.log; cd ..
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/trace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/trace.log; exit 1; }
