#!/bin/bash
# quick GPU check of selected test files: tools/gpu_r03_quick.sh TAG test_file[::test] ...
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu "$@" > gpurun_out/$T/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/$T/pytest.log | tail -12; [ $rc -eq 0 ] || grep -E "Error|assert|error" gpurun_out/$T/pytest.log | head -20; exit $rc
