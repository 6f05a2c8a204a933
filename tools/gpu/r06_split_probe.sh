#!/bin/bash
# Round 6: pass-1 timing probes (wrong outputs, timing only) per hook scale,
# back to back (tools/probe/stats_split.py) at configs 2 and 3:
# base; split = channel rounds of >= 2-round scales as separate workgroups
# storing block sums (no fold, no tail); notail; nomm (no min/max partials).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r06_split_probe
mkdir -p $O
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base0.so
for v in base split notail nomm; do
  if [ $v = base ]; then cp /tmp/base0.so $L; else cp tools/probe/ab/$v.so $L; fi
  for c in 2 3; do
    CFG=$c timeout -k 10 120 python tools/probe/stats_split.py > $O/${v}_c$c.txt 2>&1 || { cp /tmp/base0.so $L; tail -5 $O/${v}_c$c.txt; exit 1; }
    echo "== $v config $c"; grep stats $O/${v}_c$c.txt
  done
done
cp /tmp/base0.so $L
