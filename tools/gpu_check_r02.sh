#!/bin/bash
# Round-2 check: GPU parity tests, smoke(), default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -40; tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
