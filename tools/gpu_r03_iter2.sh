#!/bin/bash
# parity of the current build on the pass-2 / hook tests, then stream A/B of variants
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_core_gpu.py tests/test_pipeline_gpu.py > gpurun_out/$T/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/pytest.log | head -20; exit $rc; }
bash tools/gpu_r03_ab.sh $T "$@"
