#!/bin/bash
# A/B of variant libraries tools/probe/ab/*.so against the built one: a parity
# subset, then the default bench line twice each.  Args: variant names (no .so).
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
cp /tmp/base.so tools/probe/ab/base.so
ok="base"
for v in "$@"; do
  cp tools/probe/ab/$v.so $L
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden_case or packed or three_scales or bench_config or stats_pass" > gpurun_out/ab/$v.pytest.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 gpurun_out/ab/$v.pytest.log)"
  if [ $rc -ne 0 ]; then grep -E "FAIL|assert" gpurun_out/ab/$v.pytest.log | head -5; continue; fi
  ok="$ok $v"
done
# interleaved repetitions: base, v1, v2, ..., base, v1, v2, ...
for r in 1 2 3; do
  for v in $ok; do
    cp tools/probe/ab/$v.so $L
    timeout -k 10 120 python bench.py --no-cpu --no-e2e --steps 200 > gpurun_out/ab/$v.$r.json 2> gpurun_out/ab/$v.$r.err || { cp /tmp/base.so $L; tail -5 gpurun_out/ab/$v.$r.err; exit 1; }
  done
done
cp /tmp/base.so $L
python - <<'PY'
import json, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    agg[f.split("/")[-1].split(".")[0]].append(d["value"])
for k, v in sorted(agg.items()):
    print("%-10s mean %8.0f img/s  runs %s" % (k, sum(v) / len(v), " ".join("%.0f" % x for x in v)))
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels"]
    print("%-22s %8.0f img/s  step %5.1f us  lat %.3f ms  stats %.1f morph %.1f quant %.1f" % (f.split("/")[-1], d["value"], d["ms_per_step"] * 1e3, d["config"]["latency_ms_single_batch"], k["stats"]["us"], k["morph_finalize"]["us"], k["quant"]["us"]))
PY
