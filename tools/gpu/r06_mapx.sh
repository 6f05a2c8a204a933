#!/bin/bash
# Fused train-mode mapper (one launch per direction, in-launch granule
# exchanges): its GPU tests + the train-path tests it feeds, the config-5
# QAT line fused / staged, and a rocprofv3 kernel trace of the fused step.
# Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06_mapx}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_mapper_fused_gpu.py tests/test_train_multi_gpu.py tests/test_dist_qat_gpu.py \
  tests/test_rccl_graph_gpu.py tests/test_train_fused_gpu.py tests/test_concurrent_scales_gpu.py -x -v --timeout 200 \
  --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|error" $OUT/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --config 5 --no-cpu > $OUT/c5_fused_$i.json 2> $OUT/c5_fused_$i.err || { tail -5 $OUT/c5_fused_$i.err; exit 1; }
  MCAQ_MAPPER_FUSED=0 timeout -k 10 300 python bench.py --config 5 --no-cpu > $OUT/c5_staged_$i.json 2> $OUT/c5_staged_$i.err || { tail -5 $OUT/c5_staged_$i.err; exit 1; }
done
MCAQ_BENCH_SHARDED=1 timeout -k 10 300 python bench.py --config 5 --no-cpu > $OUT/c5_sharded.json 2> $OUT/c5_sharded.err || { tail -5 $OUT/c5_sharded.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5 -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --config 5 --steps 100 > $OUT/c5.log 2>&1) || { tail -8 $OUT/c5.log; exit 1; }
cp $OUT/c5/run_kernel_stats.csv $OUT/kernel_stats_c5.csv
python3 tools/qat_timeline.py $OUT/c5/run_kernel_trace.csv 3 > $OUT/timeline_c5.txt
for f in $OUT/c5_*.json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print(d['ms_per_step'], d['value'])")"; done
head -25 $OUT/timeline_c5.txt
