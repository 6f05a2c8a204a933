#!/bin/bash
# Round-6 final evidence of a build: full GPU tests, smoke, the default bench
# line (config 2 with CPU baseline and e2e leg), the config-5 QAT line, and
# rocprofv3 --kernel-trace --stats of config 2 (one launch at a time, k = 1;
# the pipelined default) and of config 5.  Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r06_final}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed|error" $OUT/pytest_gpu.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
timeout -k 10 300 python bench.py --config 5 > $OUT/bench_config5.json 2> $OUT/bench_config5.err || { tail -5 $OUT/bench_config5.err; exit 1; }
MCAQ_BENCH_SHARDED=1 timeout -k 10 300 python bench.py --config 5 --no-cpu > $OUT/bench_config5_sharded.json 2> $OUT/bench_config5_sharded.err || { tail -5 $OUT/bench_config5_sharded.err; exit 1; }
timeout -k 10 300 python bench.py --e2e --amp --steps 20 --warmup 3 > $OUT/bench_e2e_amp.json 2> $OUT/bench_e2e_amp.err || { tail -5 $OUT/bench_e2e_amp.err; exit 1; }
MCAQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu --steps 20 --warmup 4 > $OUT/bench_gloo_n2.json 2> $OUT/bench_gloo_n2.err || { tail -5 $OUT/bench_gloo_n2.err; exit 1; }
MCAQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --no-cpu --no-e2e --steps 20 --warmup 4 > $OUT/bench_gloo_n4.json 2> $OUT/bench_gloo_n4.err || { tail -5 $OUT/bench_gloo_n4.err; exit 1; }
MCAQ_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --config 5 --no-cpu --steps 10 --warmup 3 > $OUT/bench_gloo_n4_c5.json 2> $OUT/bench_gloo_n4_c5.err || { tail -5 $OUT/bench_gloo_n4_c5.err; exit 1; }
prof() {  # name, bench args...
  local n=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$n -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e "$@" > $OUT/$n.log 2>&1) || { tail -8 $OUT/$n.log; exit 1; }
  cp $OUT/$n/run_kernel_stats.csv $OUT/kernel_stats_$n.csv
}
prof c2_p1_k1 --pipeline 1 --launch-batches 1 --steps 100
prof c2_p3_k2 --steps 200
prof c5 --config 5 --steps 100
python3 tools/qat_timeline.py $OUT/c5/run_kernel_trace.csv 3 > $OUT/timeline_c5.txt
python3 tools/trace_analyze.py $OUT/c2_p3_k2/run_kernel_trace.csv 600 > $OUT/trace_p3_k2.txt
python3 - <<PY
import json, csv
for k in ("bench_default", "bench_config5", "bench_config5_sharded", "bench_e2e_amp", "bench_gloo_n2", "bench_gloo_n4", "bench_gloo_n4_c5"):
    d = json.loads([l for l in open("$OUT/%s.json" % k).read().splitlines() if l.startswith("{")][-1])
    r = d.get("path_roofline") or d.get("step_roofline") or {}
    print(k, d["n_gpus"], d["value"], d["ms_per_step"], r.get("frac"), (d.get("roofline") or {}).get("frac"), (d.get("cpu_baseline") or {}).get("value"), (d.get("e2e") or {}).get("value"))
for n in ("c2_p1_k1",):
    for r in csv.DictReader(open("$OUT/kernel_stats_%s.csv" % n)):
        if "mcaq" in r["Name"]:
            print("  %-58s %6s %8.2f us" % (r["Name"][:58], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
