#!/bin/bash
# m(p) plane written by pass B and read by pass 2 vs regenerated in pass 2 (interleaved)
set -o pipefail
mkdir -p gpurun_out/mplane
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in regen plane; do
    a=""; [ $v = plane ] && a="--m-plane"
    timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 400 $a > gpurun_out/mplane/$v.$r.json 2> gpurun_out/mplane/$v.$r.err || { tail -8 gpurun_out/mplane/$v.$r.err; exit 1; }
  done
done
python - <<'PY'
import json, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/mplane/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    agg[f.split("/")[-1].split(".")[0]].append(d["value"])
    print("%-16s %8.0f img/s  step %5.1f us  quant %.1f  morph %.1f" % (f.split("/")[-1], d["value"], d["ms_per_step"] * 1e3, d["kernels"]["quant"]["us"], d["kernels"]["morph_finalize"]["us"]))
for k, v in agg.items(): print(k, "mean %.0f" % (sum(v) / len(v)))
PY
