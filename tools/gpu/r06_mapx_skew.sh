#!/bin/bash
# Per-workgroup start / stage-1 end of the fused mapper forward
# (tools/probe/mapx_skew.py on the -DMCAQ_STAMPS_WG variant tools/probe/ab/wg.so).
set -o pipefail
mkdir -p gpurun_out/r06_mapx_skew
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
cp tools/probe/ab/wg.so $L
timeout -k 10 200 python tools/probe/mapx_skew.py > gpurun_out/r06_mapx_skew/skew.txt 2>&1; rc=$?
cp /tmp/base.so $L
tail -6 gpurun_out/r06_mapx_skew/skew.txt
exit $rc
