#!/bin/bash
# Round 5: launch-set parity + sweep (batches per launch x pipeline depth x morphology variant)
set -o pipefail
OUT=gpurun_out/r05_ls
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_launch_set_gpu.py > $OUT/pytest_ls.log 2>&1 || { tail -30 $OUT/pytest_ls.log; exit 1; }
tail -3 $OUT/pytest_ls.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python -u bench.py --no-cpu --no-e2e --steps 120 "$@" > $OUT/b_$n.json 2> $OUT/b_$n.err || { echo "FAIL $n"; tail -5 $OUT/b_$n.err; exit 1; }
  python - "$OUT/b_$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-14s %9.1f img/s  %7.2f us/step  path %.3f  quant %.2f us" % (sys.argv[2], d["value"], d["ms_per_step"]*1e3, d["path_roofline"]["frac"], d["kernels"]["quant"]["us"]))
PY
}
for rep in 1 2; do
  run k1d3_$rep --launch-batches 1 --pipeline 3
  run k2d3_$rep --launch-batches 2 --pipeline 3
  run k2d2_$rep --launch-batches 2 --pipeline 2
  run k3d2_$rep --launch-batches 3 --pipeline 2
  run k2d3bb_$rep --launch-batches 2 --pipeline 3 --pass-a band --pass-b batch
  run k2d3ib_$rep --launch-batches 2 --pipeline 3 --pass-b batch
  run k3d3_$rep --launch-batches 3 --pipeline 3
done
