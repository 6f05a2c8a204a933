#!/bin/bash
# Round-2 final: GPU parity tests, smoke, default bench line, bench --pipeline 1,
# rocprofv3 kernel stats at pipeline 3 and 1 (tag $1)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r02_vX}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" gpurun_out/$T/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -20 gpurun_out/$T/bench.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --no-e2e --pipeline 1 > gpurun_out/$T/bench_p1.json 2> gpurun_out/$T/bench_p1.err || { tail -20 gpurun_out/$T/bench_p1.err; exit 1; }
cd /tmp
for d in 3 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$T/p$d -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --pipeline $d > $R/gpurun_out/$T/p$d.log 2>&1 || { tail -5 $R/gpurun_out/$T/p$d.log; exit 1; }
done
cd $R && python - "$T" <<'PY'
import json, glob, csv, sys
T = sys.argv[1]
for f in sorted(glob.glob("gpurun_out/%s/bench*.json" % T)):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), "step %.1f us" % (d["ms_per_step"] * 1e3), "path", d["path_roofline"]["frac"], "quant", d["kernels"]["quant"]["us"], "stats", d["kernels"]["stats"]["us"], "morph", d["kernels"]["morph_finalize"]["us"])
    if d.get("cpu_baseline"): print("  cpu_baseline", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
    if d.get("e2e"): print("  e2e", d["e2e"].get("value"))
for f in sorted(glob.glob("gpurun_out/%s/p*/**/*kernel_stats.csv" % T, recursive=True)):
    print(f)
    for r in csv.DictReader(open(f)):
        if "mcaq" in r["Name"]:
            print("   %-60s n=%5s avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
