#!/bin/bash
# QAT: GPU tests, config-5 bench, rocprofv3 kernel stats of the same command
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/qat
cd $R
timeout -k 10 300 python -u -m pytest tests/test_qat_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qat/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/qat/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/qat/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --config 5 --no-cpu > gpurun_out/qat/bench.json 2> gpurun_out/qat/bench.err || { tail -20 gpurun_out/qat/bench.err; exit 1; }
cat gpurun_out/qat/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/qat/prof -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu > $R/gpurun_out/qat/prof.log 2>&1 || { tail -5 $R/gpurun_out/qat/prof.log; exit 1; }
cd $R && python - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/qat/prof/**/*kernel_stats.csv", recursive=True):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:14]:
        print("   %-70s n=%5s avg %8.2f us  total %8.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3))
PY
