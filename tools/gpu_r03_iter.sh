#!/bin/bash
# r03 iteration: new parity tests, then the staged schedule vs the round-2 schedule
set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py tests/test_dist_hooks.py tests/test_core_gpu.py -k "pipeline or nonfinite or sharded or cuda_kernel_parity" > gpurun_out/r03/pytest_iter.log 2>&1
rc=$?; tail -15 gpurun_out/r03/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
for v in "staged:0" "staged:64" "staged:96" "streams:0"; do
  sch=${v%%:*}; cus=${v##*:}
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 200 --warmup 20 --schedule $sch --morph-cus $cus > gpurun_out/r03/b_${sch}_${cus}.json 2> gpurun_out/r03/b_${sch}_${cus}.err || { tail -5 gpurun_out/r03/b_${sch}_${cus}.err; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/r03/b_*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['kernels']
    print("%-24s %8.0f img/s step %5.1f us frac %.3f  stats %.1f/%.1f quant %.1f/%.1f morph %.1f lat %.3f" % (f.split('/')[-1], d['value'], d['ms_per_step']*1e3, d['path_roofline']['frac'], k['stats']['us'], k['stats']['us_in_sequence'], k['quant']['us'], k['quant']['us_in_sequence'], k['morph_finalize']['us'], d['config']['latency_ms_single_batch']))
PY
