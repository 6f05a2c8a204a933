#!/bin/bash
# HBM passes alone (x cold, tools/stream_bench.py) for variant libraries in
# tools/probe/ab/, two interleaved rounds.  Usage: tools/gpu_r03_ab.sh TAG v1 v2 ...
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
for r in 1 2; do
  for v in "$@"; do
    timeout -k 10 120 python tools/stream_bench.py --lib tools/probe/ab/$v.so --tag $v > gpurun_out/$T/${v}_$r.json 2> gpurun_out/$T/${v}_$r.err || { tail -3 gpurun_out/$T/${v}_$r.err; exit 1; }
  done
done
python - "$T" <<'PY'
import json, glob, sys
for f in sorted(glob.glob("gpurun_out/%s/*.json" % sys.argv[1])):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print("%-22s stats %6.2f us (%.3f)  quant %6.2f us (%.3f)  back-to-back %6.2f us/step (path %.3f)" % (f.split("/")[-1][:-5], d["stats"]["us"], d["stats"]["frac"], d["quant"]["us"], d["quant"]["frac"], d["stats+quant back to back"]["us_per_step"], d["stats+quant back to back"]["path_frac_if_hidden"]))
PY
