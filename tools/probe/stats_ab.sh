#!/bin/bash
# per-scale pass-1 timing (tools/probe/stats_split.py) for variant libraries tools/probe/ab/<v>.so
set -o pipefail
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
mkdir -p gpurun_out/sab
for v in base "$@"; do
  [ "$v" = base ] && cp /tmp/base.so $L || cp tools/probe/ab/$v.so $L
  echo "== $v"
  timeout -k 10 120 python tools/probe/stats_split.py > gpurun_out/sab/$v.log 2>&1 || { cp /tmp/base.so $L; tail -5 gpurun_out/sab/$v.log; exit 1; }
  grep -E "stats|quant" gpurun_out/sab/$v.log
done
cp /tmp/base.so $L
