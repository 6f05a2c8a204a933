#!/bin/bash
# batches in flight x HIP hardware queues per process (interleaved repetitions)
set -o pipefail
mkdir -p gpurun_out/queues
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "3 4" "4 8" "5 8" "6 8" "4 4"; do set -- $cfg
    GPU_MAX_HW_QUEUES=$2 timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 300 --pipeline $1 > gpurun_out/queues/d$1_q$2.$r.json 2> gpurun_out/queues/d$1_q$2.$r.err || { tail -8 gpurun_out/queues/d$1_q$2.$r.err; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/queues/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print("%-22s %8.0f img/s  step %5.1f us" % (f.split("/")[-1], d["value"], d["ms_per_step"] * 1e3))
PY
