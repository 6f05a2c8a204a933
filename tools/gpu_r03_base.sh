#!/bin/bash
# r03 baseline on a fresh box: full GPU tests, smoke, bench staged vs streams
# (400 and 20 steps), rocprofv3 kernel stats of the default bench.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_base}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/$T/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -2 gpurun_out/$T/smoke.log
for v in "staged:400" "streams:400" "staged:20" "streams:20" "staged:400"; do
  sch=${v%%:*}; n=${v##*:}
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps $n --warmup 20 --schedule $sch > gpurun_out/$T/b_${sch}_${n}_$RANDOM.json 2> gpurun_out/$T/b_${sch}_${n}.err || { tail -5 gpurun_out/$T/b_${sch}_${n}.err; exit 1; }
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e > $R/gpurun_out/$T/prof.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof.log; exit 1; }
cd $R && python tools/summarize_r03.py gpurun_out/$T
