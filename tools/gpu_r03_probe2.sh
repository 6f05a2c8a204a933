#!/bin/bash
# r03 probes: CU-mask bandwidth / graph-branch concurrency / host API costs,
# Infinity-Cache residency of x between the two passes, kernel trace of the
# default (streams) schedule, staged schedule with CU masks.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_probe2}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 120 ./tools/probe/mall_probe > gpurun_out/$T/mall_probe.txt 2>&1; rc=$?; cat gpurun_out/$T/mall_probe.txt; [ $rc -eq 0 ] || exit $rc
for v in "streams:0"; do
  sch=${v%%:*}; cus=${v##*:}
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 400 --warmup 20 --schedule $sch --morph-cus $cus > gpurun_out/$T/b_${sch}_${cus}.json 2> gpurun_out/$T/b_${sch}_${cus}.err || { tail -5 gpurun_out/$T/b_${sch}_${cus}.err; exit 1; }
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --schedule streams > $R/gpurun_out/$T/prof.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof.log; exit 1; }
cd $R && python tools/summarize_r03.py gpurun_out/$T && python tools/trace_analyze.py gpurun_out/$T/prof/run_kernel_trace.csv 800
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/qat -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu --steps 20 --warmup 3 > $R/gpurun_out/$T/qat.log 2>&1 || { tail -5 $R/gpurun_out/$T/qat.log; exit 1; }
cd $R && tail -1 gpurun_out/$T/qat.log | cut -c1-400
