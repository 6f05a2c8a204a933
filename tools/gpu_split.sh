#!/bin/bash
# --schedule split vs the default multi-stream schedule (interleaved repetitions)
set -o pipefail
mkdir -p gpurun_out/split
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "streams 3" "split 2" "split 3" "split 4"; do set -- $cfg
    timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 --schedule $1 --lookahead $2 > gpurun_out/split/$1_$2.$r.json 2> gpurun_out/split/$1_$2.$r.err || { tail -8 gpurun_out/split/$1_$2.$r.err; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/split/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print("%-24s %8.0f img/s  step %5.1f us  host %.1f us" % (f.split("/")[-1], d["value"], d["ms_per_step"] * 1e3, d["config"]["host_enqueue_us_per_step"]))
PY
