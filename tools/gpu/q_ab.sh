#!/bin/bash
# GPU_MAX_HW_QUEUES 4 vs 8 (and 6) at pipeline depth 3, interleaved rounds.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-q_ab}
mkdir -p $R/gpurun_out/$T
cd $R
for r in 1 2 3 4 5; do
  for q in 4 8 6; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 > gpurun_out/$T/b_q${q}_$r.json 2> gpurun_out/$T/b_q${q}_$r.err || { tail -5 gpurun_out/$T/b_q${q}_$r.err; exit 1; }
  done
done
python - <<PY
import json, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/$T/b_q*.json")):
    d = json.load(open(f))
    agg[f.split("/")[-1].split("_")[1]].append(d["value"])
for k, v in sorted(agg.items()):
    print("%-4s mean %8.0f img/s  min %8.0f  max %8.0f  runs %s" % (k, sum(v) / len(v), min(v), max(v), " ".join("%.0f" % x for x in v)))
PY
