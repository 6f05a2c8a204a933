#!/bin/bash
# r03: 4-stream staged pipeline as captured HIP graphs: pipeline tests, staged vs streams A/B, rocprof of staged
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_graph}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_pipeline_gpu.py > gpurun_out/$T/pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/$T/pytest.log | tail -8; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/$T/pytest.log | head -30; exit $rc; }
for v in "staged:20" "streams:20" "staged:400" "streams:400" "staged:20" "staged:400"; do
  sch=${v%%:*}; n=${v##*:}
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps $n --warmup 20 --schedule $sch > gpurun_out/$T/b_${sch}_${n}_$RANDOM.json 2> gpurun_out/$T/b_${sch}_${n}.err || { tail -5 gpurun_out/$T/b_${sch}_${n}.err; exit 1; }
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --schedule staged --steps 400 > $R/gpurun_out/$T/prof.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof.log; exit 1; }
cd $R && python tools/summarize_r03.py gpurun_out/$T
