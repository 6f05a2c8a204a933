#!/bin/bash
# A/B of variant libraries tools/probe/ab/*.so on the config-5 QAT step: the
# fused-launch GPU tests, then the config-5 line 3x interleaved (base first).
# Args: variant names (no .so).  Out: gpurun_out/ab_c5/.
set -o pipefail
mkdir -p gpurun_out/ab_c5
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
cp /tmp/base.so tools/probe/ab/base.so
ok="base"
for v in "$@"; do
  cp tools/probe/ab/$v.so $L
  timeout -k 10 300 python -u -m pytest tests/test_mapper_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_c5/$v.pytest.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 gpurun_out/ab_c5/$v.pytest.log)"
  if [ $rc -ne 0 ]; then cp /tmp/base.so $L; exit $rc; fi
  ok="$ok $v"
done
for r in 1 2 3; do
  for v in $ok; do
    cp tools/probe/ab/$v.so $L
    timeout -k 10 200 python bench.py --config 5 --no-cpu > gpurun_out/ab_c5/$v.$r.json 2> gpurun_out/ab_c5/$v.$r.err || { cp /tmp/base.so $L; tail -5 gpurun_out/ab_c5/$v.$r.err; exit 1; }
  done
done
cp /tmp/base.so $L
for f in gpurun_out/ab_c5/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print(d['ms_per_step'])")"; done
