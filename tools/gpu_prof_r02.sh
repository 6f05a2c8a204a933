#!/bin/bash
# bench lines (default and --pipeline 1) + rocprofv3 kernel stats of both commands. Tag = $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r02_vX}
mkdir -p $R/gpurun_out/prof_$T
cd $R
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/prof_$T/bench.json 2> gpurun_out/prof_$T/bench.err || { tail -20 gpurun_out/prof_$T/bench.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --no-e2e --pipeline 1 > gpurun_out/prof_$T/bench_p1.json 2> gpurun_out/prof_$T/bench_p1.err || { tail -20 gpurun_out/prof_$T/bench_p1.err; exit 1; }
cd /tmp
for d in 3 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T/p$d -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --pipeline $d > $R/gpurun_out/prof_$T/p$d.log 2>&1 || { tail -5 $R/gpurun_out/prof_$T/p$d.log; exit 1; }
done
cd $R && python - <<'PY'
import json, glob, csv, os
T = os.environ.get("T_TAG")
for f in sorted(glob.glob("gpurun_out/prof_*/bench*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), "step %.1f us" % (d["ms_per_step"] * 1e3), "path", d["path_roofline"]["frac"], "quant", d["kernels"]["quant"]["us"], "stats", d["kernels"]["stats"]["us"], "morph", d["kernels"]["morph_finalize"]["us"])
for f in sorted(glob.glob("gpurun_out/prof_*/p*/**/*kernel_stats.csv", recursive=True)):
    print(f)
    for r in csv.DictReader(open(f)):
        if "mcaq" in r["Name"]:
            print("   %-60s n=%5s avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
