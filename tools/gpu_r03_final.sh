#!/bin/bash
# r03 validation of a build: full GPU tests, smoke, default bench (20 / 400
# steps), pipeline-1 bench, rocprofv3 kernel stats at pipeline 1 and 3, PMC
# HBM traffic.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_final}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/$T/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -2 gpurun_out/$T/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/$T/b_default.json 2> gpurun_out/$T/b_default.err || { tail -5 gpurun_out/$T/b_default.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 20 > gpurun_out/$T/b_steps20.json 2> gpurun_out/$T/b_steps20.err || { tail -5 gpurun_out/$T/b_steps20.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu --no-e2e --pipeline 1 > gpurun_out/$T/b_pipeline1.json 2> gpurun_out/$T/b_pipeline1.err || { tail -5 gpurun_out/$T/b_pipeline1.err; exit 1; }
cd /tmp
for p in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof_p$p -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --pipeline $p > $R/gpurun_out/$T/prof_p$p.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof_p$p.log; exit 1; }
done
cd $R && bash tools/pmc_traffic.sh > gpurun_out/$T/pmc.log 2>&1 || { tail -5 gpurun_out/$T/pmc.log; exit 1; }
cp gpurun_out/pmc_summary.json gpurun_out/$T/pmc_summary.json
python tools/summarize_r03.py gpurun_out/$T
