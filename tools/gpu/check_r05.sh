#!/bin/bash
# Round-5 validation of a build: full GPU tests, smoke, the default bench
# line (CPU baseline and e2e leg included) and a 20-step line.  Tag $1 ->
# gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r05_check}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/$T/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -2 gpurun_out/$T/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err || { tail -5 gpurun_out/$T/bench_default.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 20 --warmup 5 > gpurun_out/$T/b_steps20.json 2> gpurun_out/$T/b_steps20.err || { tail -5 gpurun_out/$T/b_steps20.err; exit 1; }
python - <<PY
import json
for k in ("bench_default", "b_steps20"):
    d = json.load(open("gpurun_out/$T/%s.json" % k))
    print(k, d["value"], d["ms_per_step"], d["path_roofline"]["frac"], d["roofline"]["frac"], (d.get("cpu_baseline") or {}).get("value"), (d.get("e2e") or {}).get("value"))
PY
