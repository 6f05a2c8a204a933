#!/bin/bash
# pass-1 cost split: the built library vs probe builds without the ATen tail
# pass and/or without the min/max partials (timing only), per scale, back to back
set -o pipefail
mkdir -p gpurun_out/stats_probe
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
for v in base ${VARIANTS:-notail nomm notail_nomm}; do
  if [ $v = base ]; then cp /tmp/base.so $L; else cp tools/probe/ab/$v.so $L; fi
  echo "== $v"
  timeout -k 10 120 python tools/probe/stats_split.py > gpurun_out/stats_probe/$v.txt 2>&1 || { cp /tmp/base.so $L; tail -5 gpurun_out/stats_probe/$v.txt; exit 1; }
  grep -E "stats|quant" gpurun_out/stats_probe/$v.txt
done
cp /tmp/base.so $L
