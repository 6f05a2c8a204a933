#!/bin/bash
# Round 6: configs 3 and 4 on the current build - bench lines at 1 and 2
# batches per launch set (k), and rocprofv3 --kernel-trace --stats of one
# launch at a time (p1, k = 1).  Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r06_configs}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
for c in 3 4; do
  for k in 1 2; do
    timeout -k 10 400 python bench.py --config $c --no-cpu --no-e2e --launch-batches $k > $OUT/b_c${c}_k$k.json 2> $OUT/b_c${c}_k$k.err || { tail -5 $OUT/b_c${c}_k$k.err; exit 1; }
  done
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c${c}_p1 -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu --no-e2e --pipeline 1 --launch-batches 1 --steps 60 > $OUT/c${c}_p1.log 2>&1) || { tail -8 $OUT/c${c}_p1.log; exit 1; }
  cp $OUT/c${c}_p1/run_kernel_stats.csv $OUT/kernel_stats_c${c}_p1_k1.csv
done
python3 - <<PY
import json, csv
for c in (3, 4):
    for k in (1, 2):
        d = json.load(open("$OUT/b_c%d_k%d.json" % (c, k)))
        print("config", c, "k", k, round(d["value"]), d["ms_per_step"], d["path_roofline"]["frac"], d["roofline"]["frac"])
    for r in csv.DictReader(open("$OUT/kernel_stats_c%d_p1_k1.csv" % c)):
        if "mcaq" in r["Name"]:
            print("  %-58s %6s %8.2f us" % (r["Name"][:58], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
