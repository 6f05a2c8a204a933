#!/bin/bash
# Round 6: pass-1 cross-row min/max on v_permlane16/32_swap (plane), tail
# items pixel-major (tailpx), both (planetail); + PPL 4 for >= 3 rounds
# (planer4p4).  Parity of the combined variant first (stats / min-max tests
# with the variant library in place), then interleaved A/B at configs 2, 3.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
L=mcaq_yolo_amd/lib/libmcaq_hip.so
mkdir -p gpurun_out/r06_ab_stats2
cp $L /tmp/base0.so
cp tools/probe/ab/planetail.so $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_core_gpu.py -x -q -k "stats or minmax or golden or nonfinite" --timeout 200 --timeout-method thread > gpurun_out/r06_ab_stats2/pytest_planetail.log 2>&1
rc=$?; cp /tmp/base0.so $L; tail -3 gpurun_out/r06_ab_stats2/pytest_planetail.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash tools/gpu/ab.sh r06_ab_stats2_c2 plane tailpx planetail planer4p4 &&
ROUNDS=2 BENCH_ARGS="--config 3 --launch-batches 1" bash tools/gpu/ab.sh r06_ab_stats2_c3 plane tailpx planetail planer4p4
