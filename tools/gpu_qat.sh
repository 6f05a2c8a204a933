#!/bin/bash
# QAT GPU tests only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_qat_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_qat.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_qat.log | tail -30; [ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_qat.log; exit $rc; }
