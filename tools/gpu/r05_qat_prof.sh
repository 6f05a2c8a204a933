#!/bin/bash
# Round 5: QAT step (config 5) kernel timeline (rocprofv3 kernel trace of the
# graph-replayed step) + bench lines; tag $1.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r05_qat}
OUT=gpurun_out/$T
mkdir -p $OUT
if [ -n "$QTESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $QTESTS > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for v in fused torch; do
  ex=""; [ $v = torch ] && ex="--torch-optim"
  timeout -k 10 200 python -u bench.py --config 5 --no-cpu --steps 200 $ex > $OUT/b_c5_$v.json 2> $OUT/b_c5_$v.err || { tail -10 $OUT/b_c5_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/b_c5_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --config 5 --no-cpu --steps 30 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python tools/qat_timeline.py $f > $OUT/timeline.txt && head -3 $OUT/timeline.txt && tail -1 $OUT/timeline.txt
