#!/bin/bash
# Round-6 in-launch exchanges (fused mapper, one-launch ClipAdamW, the MLP
# backward's in-launch parameter reduction): their GPU
# tests + the train-path tests they feed, config-5 QAT lines for every on/off
# combination (interleaved), a rocprofv3 kernel trace of the default step and
# the fused mapper's stage stamps.  Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06_fuse}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_mapper_fused_gpu.py tests/test_optim_gpu.py tests/test_train_multi_gpu.py \
  tests/test_dist_qat_gpu.py tests/test_rccl_graph_gpu.py tests/test_train_fused_gpu.py tests/test_concurrent_scales_gpu.py \
  tests/test_qat_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "passed|failed|error" $OUT/pytest.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
for i in 1 2; do
  for v in "1 1 1" "1 1 0" "1 0 1" "0 1 1" "0 0 0"; do
    set -- $v
    n=c5_m$1_o$2_h$3_$i
    MCAQ_MAPPER_FUSED=$1 MCAQ_ADAMW_ONE_LAUNCH=$2 MCAQ_HEAD_FUSED=$3 timeout -k 10 300 python bench.py --config 5 --no-cpu > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
  done
done
MCAQ_BENCH_SHARDED=1 timeout -k 10 300 python bench.py --config 5 --no-cpu > $OUT/c5_sharded.json 2> $OUT/c5_sharded.err || { tail -5 $OUT/c5_sharded.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5 -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-e2e --config 5 --steps 100 > $OUT/c5.log 2>&1) || { tail -8 $OUT/c5.log; exit 1; }
cp $OUT/c5/run_kernel_stats.csv $OUT/kernel_stats_c5.csv
python3 tools/qat_timeline.py $OUT/c5/run_kernel_trace.csv 3 > $OUT/timeline_c5.txt
if [ -f mcaq_yolo_amd/lib/libmcaq_hip_stamps.so ]; then
  timeout -k 10 240 python tools/probe/train_stamps.py > $OUT/train_stamps.txt 2>&1 || { tail -5 $OUT/train_stamps.txt; exit 1; }
  tail -10 $OUT/train_stamps.txt
fi
for f in $OUT/c5_*.json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print(d['ms_per_step'], d['value'])")"; done
head -25 $OUT/timeline_c5.txt
