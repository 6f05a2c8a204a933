#!/bin/bash
# QAT GPU tests + QAT bench (config 5, graph and eager) + rocprof kernel stats of the QAT step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_qat_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qat.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_qat.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_qat.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --config 5 --steps 30 --warmup 5 > gpurun_out/bench_qat.json 2> gpurun_out/bench_qat.err || { tail -30 gpurun_out/bench_qat.err; exit 1; }
cat gpurun_out/bench_qat.json
timeout -k 10 300 python bench.py --config 5 --steps 30 --warmup 5 --eager --no-cpu > gpurun_out/bench_qat_eager.json 2> gpurun_out/bench_qat_eager.err || { tail -30 gpurun_out/bench_qat_eager.err; exit 1; }
cut -c1-400 gpurun_out/bench_qat_eager.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_qat -o run --output-format csv -- python3 $R/bench.py --config 5 --steps 20 --warmup 3 --no-cpu > $R/gpurun_out/prof_qat.log 2>&1 || { tail -20 $R/gpurun_out/prof_qat.log; exit 1; }
cut -c1-160 $R/gpurun_out/prof_qat/run_kernel_stats.csv | head -25
