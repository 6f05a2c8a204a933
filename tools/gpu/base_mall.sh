#!/bin/bash
# Round-4 re-entry: the concurrent-scales tests (report only), the Infinity
# Cache probe (tools/probe/mall_probe, built on the CPU side), then the full
# validation of tools/gpu/check.sh with the QAT bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r04_base}
cd $R
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_concurrent_scales_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_conc.log 2>&1
echo "concurrent tests rc=$?"; grep -E "passed|failed|Error|assert" gpurun_out/$T/pytest_conc.log | tail -8
timeout -k 10 120 ./tools/probe/mall_probe > gpurun_out/$T/mall_probe.txt 2>&1 || { tail -5 gpurun_out/$T/mall_probe.txt; exit 1; }
cat gpurun_out/$T/mall_probe.txt
timeout -k 10 200 python bench.py --config 5 --no-cpu --steps 100 > gpurun_out/$T/b_config5.json 2> gpurun_out/$T/b_config5.err || { tail -5 gpurun_out/$T/b_config5.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/$T/b_config5.json')); print('config5', d['value'], d['ms_per_step'], d['mapper'])"
bash tools/gpu/check.sh $T
