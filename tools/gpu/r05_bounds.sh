#!/bin/bash
# Round 5: measured structure of the config-2 step with launch sets: rocprofv3
# kernel stats one launch at a time (p1, 1 and 2 batches per launch), the
# pipelined default (p3, 2 batches per launch) with its kernel trace analysed
# for concurrency, and the bound probe (full / streaming-only / morphology-only)
# at 1 and 2 batches per launch.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
T=${1:-r05_bounds}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
prof() {  # name, bench args...
  local n=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$n -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e "$@" > $OUT/$n.log 2>&1) || { tail -8 $OUT/$n.log; exit 1; }
  cp $OUT/$n/run_kernel_stats.csv $OUT/kernel_stats_$n.csv
  python3 - $OUT/kernel_stats_$n.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "mcaq" in n:
        print("   %-60s calls %6s  avg %8.2f us" % (n[:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
echo "== p1 k1"; prof p1_k1 --pipeline 1 --launch-batches 1 --steps 100
echo "== p1 k2"; prof p1_k2 --pipeline 1 --launch-batches 2 --steps 100
echo "== p3 k2 (default)"; prof p3_k2 --steps 200
python3 $R/tools/trace_analyze.py $OUT/p3_k2/run_kernel_trace.csv 600 > $OUT/trace_p3_k2.txt && cat $OUT/trace_p3_k2.txt
for k in 1 2; do
  echo "== bound probe k=$k"
  timeout -k 10 300 python3 -u $R/tools/probe/bound_probe.py $k > $OUT/bound_k$k.txt 2>&1 || { tail -5 $OUT/bound_k$k.txt; exit 1; }
  cat $OUT/bound_k$k.txt
done
