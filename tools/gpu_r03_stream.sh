#!/bin/bash
# HBM passes alone (x cold), current build vs variant libraries
set -o pipefail
mkdir -p gpurun_out/r03/stream
export TMPDIR=/tmp
for v in cur "$@"; do
  lib=mcaq_yolo_amd/lib/libmcaq_hip.so; [ $v = cur ] || lib=tools/probe/ab/$v.so
  timeout -k 10 120 python tools/stream_bench.py --lib $lib --tag $v > gpurun_out/r03/stream/$v.json 2> gpurun_out/r03/stream/$v.err || { tail -3 gpurun_out/r03/stream/$v.err; exit 1; }
  cat gpurun_out/r03/stream/$v.json
done
