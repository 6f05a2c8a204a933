#!/bin/bash
# A/B: pass-1 nontemporal loads of x (variant library built with -DMCAQ_STATS_NTL)
set -o pipefail
mkdir -p gpurun_out
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
for rep in a b; do
  cp /tmp/base.so $L
  timeout -k 10 180 python bench.py --no-cpu --steps 100 > gpurun_out/ntl0$rep.json 2>gpurun_out/ntl0$rep.err || exit 1
  cp tools/probe/libmcaq_hip_ntl.so $L
  timeout -k 10 180 python bench.py --no-cpu --steps 100 > gpurun_out/ntl1$rep.json 2>gpurun_out/ntl1$rep.err || exit 1
done
cp /tmp/base.so $L
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/ntl*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), d["kernels"]["stats"]["us"], d["kernels"]["quant"]["us"])
PY
