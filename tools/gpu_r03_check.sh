#!/bin/bash
# r03 re-entry check: full GPU tests, smoke, default bench (20/400 steps), config-5 bench + rocprof.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_check}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/$T/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -2 gpurun_out/$T/smoke.log
for n in 20 400; do
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps $n --warmup 20 > gpurun_out/$T/b_streams_$n.json 2> gpurun_out/$T/b_streams_$n.err || { tail -5 gpurun_out/$T/b_streams_$n.err; exit 1; }
done
timeout -k 10 300 python bench.py --config 5 --no-cpu --steps 50 --warmup 5 > gpurun_out/$T/bench5.json 2> gpurun_out/$T/bench5.err || { tail -20 gpurun_out/$T/bench5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/$T/bench5.json').read().strip().splitlines()[-1]); print('config5', d['value'], 'img/s', d['ms_per_step'], 'ms/step', d.get('kernels'))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof5 -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu --steps 20 --warmup 3 > $R/gpurun_out/$T/prof5.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof5.log; exit 1; }
cd $R && python tools/summarize_r03.py gpurun_out/$T
