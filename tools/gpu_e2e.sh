#!/bin/bash
# e2e path: NMS + MCAQYOLO GPU tests, then the end-to-end bench (fp32 and bf16 network).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_e2e_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_e2e.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_e2e.log | tail -20; [ $rc -eq 0 ] || { tail -80 gpurun_out/pytest_e2e.log; exit $rc; }
timeout -k 10 300 python bench.py --e2e --steps 20 --warmup 3 > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err || { tail -30 gpurun_out/bench_e2e.err; exit 1; }
cat gpurun_out/bench_e2e.json
timeout -k 10 300 python bench.py --e2e --amp --steps 20 --warmup 3 > gpurun_out/bench_e2e_amp.json 2> gpurun_out/bench_e2e_amp.err || { tail -30 gpurun_out/bench_e2e_amp.err; exit 1; }
cat gpurun_out/bench_e2e_amp.json
