#!/bin/bash
# NMS + e2e GPU tests, e2e bench line, rocprof of the e2e leg
set -o pipefail
mkdir -p gpurun_out/nms
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_e2e_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/nms/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/nms/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/nms/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --e2e --steps 20 --warmup 3 > gpurun_out/nms/e2e.json 2> gpurun_out/nms/e2e.err || { tail -8 gpurun_out/nms/e2e.err; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/nms/prof -o run --output-format csv -- python3 $R/bench.py --e2e --steps 20 --warmup 3 > $R/gpurun_out/nms/prof.log 2>&1 || { tail -5 $R/gpurun_out/nms/prof.log; exit 1; }
cd $R && python - <<'PY'
import json, glob, csv
d = json.loads(open("gpurun_out/nms/e2e.json").read().strip().splitlines()[-1]); c = d["config"]
print("e2e %8.0f img/s  step %6.3f ms  net %6.3f ms  hooks+nms %6.3f ms det/img %.1f" % (d["value"], d["ms_per_step"], c["network_only_ms_per_step"], c["mcaq_hooks_and_nms_ms_per_step"], c["detections_per_image"]))
for f in glob.glob("gpurun_out/nms/prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mcaq" in r["Name"]:
            print("   %-60s n=%5s avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
