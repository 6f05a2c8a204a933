#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/e2e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python bench.py --e2e --steps 20 --warmup 3 --find > gpurun_out/e2e/fuse_find.json 2> gpurun_out/e2e/fuse_find.err || { tail -8 gpurun_out/e2e/fuse_find.err; exit 1; }
timeout -k 10 400 python bench.py --e2e --steps 20 --warmup 3 --find --amp > gpurun_out/e2e/fuse_find_amp.json 2> gpurun_out/e2e/fuse_find_amp.err || { tail -8 gpurun_out/e2e/fuse_find_amp.err; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/e2e/prof -o run --output-format csv -- python3 $R/bench.py --e2e --steps 20 --warmup 3 > $R/gpurun_out/e2e/prof.log 2>&1 || { tail -5 $R/gpurun_out/e2e/prof.log; exit 1; }
cd $R && python - <<'PY'
import json, glob, csv
for f in sorted(glob.glob("gpurun_out/e2e/fuse_find*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); c = d["config"]
    print("%-20s %8.0f img/s  step %6.3f ms  net %6.3f ms  hooks+nms %6.3f ms" % (f.split("/")[-1], d["value"], d["ms_per_step"], c["network_only_ms_per_step"], c["mcaq_hooks_and_nms_ms_per_step"]))
for f in glob.glob("gpurun_out/e2e/prof/**/*kernel_stats.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("total kernel time %.1f ms" % (tot / 1e6))
    for r in rows[:16]:
        print("   %-80s n=%5s avg %8.2f us  total %8.1f us" % (r["Name"][:80], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3))
PY
