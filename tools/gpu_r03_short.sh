#!/bin/bash
# r03 short validation: full GPU tests, smoke, default bench, 20-step bench.  Tag $1.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r03_short}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/$T/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -2 gpurun_out/$T/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/$T/b_default.json 2> gpurun_out/$T/b_default.err || { tail -5 gpurun_out/$T/b_default.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 20 > gpurun_out/$T/b_steps20.json 2> gpurun_out/$T/b_steps20.err || { tail -5 gpurun_out/$T/b_steps20.err; exit 1; }
python tools/summarize_r03.py gpurun_out/$T
