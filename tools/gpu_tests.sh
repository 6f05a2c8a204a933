#!/bin/bash
# GPU parity tests only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -30; [ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
