set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_qat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qat.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_qat.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_qat.log | head -30; exit $rc; }
timeout -k 10 200 python tools/prof_stats.py 2 > gpurun_out/prof_stats.txt 2>&1; rc=$?; cat gpurun_out/prof_stats.txt; exit $rc
