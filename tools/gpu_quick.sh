#!/bin/bash
# Short GPU session: parity tests + kernel diagnostics.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
cd $GRAFT_REPO_ROOT/tools && timeout -k 10 120 python prof_stages.py 2 > ../gpurun_out/stages.log 2>&1; cat ../gpurun_out/stages.log
cd $GRAFT_REPO_ROOT && timeout -k 10 120 python tools/prof_morph_stamps.py 2 > gpurun_out/stamps.log 2>&1; head -16 gpurun_out/stamps.log
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
