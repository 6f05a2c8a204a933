set -o pipefail
O=gpurun_out/r06_split_b16; mkdir -p $O
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base0.so
for v in base split notail; do
  if [ $v = base ]; then cp /tmp/base0.so $L; else cp tools/probe/ab/$v.so $L; fi
  BATCH=16 CFG=2 timeout -k 10 120 python tools/probe/stats_split.py > $O/${v}_b16.txt 2>&1 || { cp /tmp/base0.so $L; tail -5 $O/${v}_b16.txt; exit 1; }
  echo "== $v bs16"; grep stats $O/${v}_b16.txt
done
cp /tmp/base0.so $L
