#!/bin/bash
# r03: Infinity-Cache probe + baseline bench of the round-2 build vs the current build
set -o pipefail
mkdir -p gpurun_out/r03
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/new.so
timeout -k 10 120 ./tools/probe/mall_probe > gpurun_out/r03/mall_probe.txt 2>&1 && cat gpurun_out/r03/mall_probe.txt || exit 1
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then cp tools/probe/ab/base_r02.so $L; else cp /tmp/new.so $L; fi
    timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 400 --warmup 20 > gpurun_out/r03/bench_${v}_$r.json 2> gpurun_out/r03/bench_${v}_$r.err || { cp /tmp/new.so $L; tail -5 gpurun_out/r03/bench_${v}_$r.err; exit 1; }
  done
done
cp /tmp/new.so $L
timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 20 --warmup 5 > gpurun_out/r03/bench_new20.json 2> gpurun_out/r03/bench_new20.err || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/r03/bench_*.json')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['kernels']
    print("%-24s %8.0f img/s step %5.1f us frac %.3f  stats %.1f morph %.1f quant %.1f" % (f.split('/')[-1], d['value'], d['ms_per_step']*1e3, d['path_roofline']['frac'], k['stats']['us'], k['morph_finalize']['us'], k['quant']['us']))
PY
