#!/bin/bash
# Infinity-Cache (MALL) reuse experiment: pass-1 NT vs plain loads x batches in flight.
set -o pipefail
mkdir -p gpurun_out/mall
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
for v in nt plain; do
  if [ $v = plain ]; then cp tools/probe/libmcaq_hip_plain.so $L; else cp /tmp/base.so $L; fi
  for d in 1 2 3; do
    for n in 3 6; do
      timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 60 --pipeline $d --inputs $n > gpurun_out/mall/${v}_d${d}_n${n}.json 2>gpurun_out/mall/${v}_d${d}_n${n}.err || { cp /tmp/base.so $L; tail -5 gpurun_out/mall/${v}_d${d}_n${n}.err; exit 1; }
    done
  done
done
cp /tmp/base.so $L
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/mall/*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print("%-28s %8.0f img/s  step %.1f us  quant-in-context %.1f us  lat %.3f ms" % (f.split('/')[-1], d["value"], d["ms_per_step"]*1e3, d["roofline"]["us_per_launch"], d["config"]["latency_ms_single_batch"]))
PY
