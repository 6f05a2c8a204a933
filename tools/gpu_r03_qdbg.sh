#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_qdbg
timeout -k 10 300 python -u -m pytest -x -s -q --timeout 200 --timeout-method thread -m gpu "tests/test_train_fused_gpu.py::test_fused_train_step_matches_torch_path" > gpurun_out/r03_qdbg/pytest.log 2>&1; rc=$?; grep -E "err|passed|failed" gpurun_out/r03_qdbg/pytest.log | tail -50; exit $rc
