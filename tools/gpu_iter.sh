#!/bin/bash
# One iteration: GPU parity tests, morph stage stamps, bench at pipeline 1 and 3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 120 python tools/prof_morph_stamps.py 2 > gpurun_out/stamps.log 2>&1 || { tail gpurun_out/stamps.log; exit 1; }
grep -E "scale|B |M binar|M sobel|E blur" gpurun_out/stamps.log
for d in 1 3; do
  timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu --pipeline $d > gpurun_out/bench_p$d.json 2> gpurun_out/bench_p$d.err || { tail -20 gpurun_out/bench_p$d.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_p$d.json'));k=d['kernels'];print('pipeline',$d,d['value'],d['ms_per_step'],d['roofline']['frac'],d['config']['latency_ms_single_batch'],{n:v['us'] for n,v in k.items()})"
done
