#!/bin/bash
# r03: fused train-mode kernels: parity tests, config-5 bench, rocprof stats (tag $1)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_qat}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_train_fused_gpu.py tests/test_qat_gpu.py > gpurun_out/$T/pytest.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -3; [ $rc -eq 0 ] || { grep -E "Error|assert|max err|FAIL" gpurun_out/$T/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --config 5 --no-cpu --steps 50 --warmup 5 > gpurun_out/$T/bench5.json 2> gpurun_out/$T/bench5.err || { tail -20 gpurun_out/$T/bench5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/$T/bench5.json').read().strip().splitlines()[-1]); print('config5', d['value'], 'img/s', d['ms_per_step'], 'ms/step')"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/prof5 -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu --steps 20 --warmup 3 > $R/gpurun_out/$T/prof5.log 2>&1 || { tail -5 $R/gpurun_out/$T/prof5.log; exit 1; }
cd $R && python tools/qat_stats.py gpurun_out/$T/prof5/run_kernel_stats.csv
