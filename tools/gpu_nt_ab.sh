#!/bin/bash
# A/B of the quant kernel's nontemporal loads/stores (MCAQ_QUANT_NT bitmask).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in a b; do for cfg in 2 3; do for nt in 0 1 2 3; do
  MCAQ_QUANT_NT=$nt timeout -k 10 180 python bench.py --no-cpu --config $cfg --steps 100 > gpurun_out/nt${nt}${rep}_c$cfg.json 2>gpurun_out/nt${nt}${rep}_c$cfg.err || exit 1
done; done; done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/nt*_c*.json"), key=lambda f: (f[-6:], f)):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), d["roofline"]["us_per_launch"], d["roofline"]["frac"], d["kernels"]["stats"]["us"])
PY
