#!/bin/bash
# bench lines for configs 3 and 4 (hook path) and config 5 (QAT), plus the gloo rehearsal of N=2
set -o pipefail
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
for c in 3 4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-e2e > gpurun_out/configs/c$c.json 2> gpurun_out/configs/c$c.err || { tail -8 gpurun_out/configs/c$c.err; exit 1; }
done
timeout -k 10 300 python bench.py --config 5 --no-cpu > gpurun_out/configs/c5.json 2> gpurun_out/configs/c5.err || { tail -8 gpurun_out/configs/c5.err; exit 1; }
python - <<'PY'
import json
for c in (3, 4, 5):
    d = json.loads(open("gpurun_out/configs/c%d.json" % c).read().strip().splitlines()[-1])
    pr = d.get("path_roofline") or d.get("step_roofline")
    print(c, d["config"]["workload"][:60], "%.0f img/s" % d["value"], "step %.1f us" % (d["ms_per_step"] * 1e3),
          "path/step frac", pr["frac"], "roofline", d["roofline"]["frac"], d["roofline"]["us_per_launch"])
PY
