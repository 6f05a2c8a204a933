#!/bin/bash
# A/B of QAT kernel variants tools/probe/ab/<v>.so: QAT GPU tests on the built
# library, then the config-5 bench's per-dispatch kernel times per variant.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/qab
L=mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
[ -n "$SKIPTEST" ] || timeout -k 10 300 python -u -m pytest tests/test_qat_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qab/pytest.log 2>&1
rc=$?; [ -n "$SKIPTEST" ] || tail -1 gpurun_out/qab/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/qab/pytest.log | head -20; exit $rc; }
for v in "$@"; do
  cp tools/probe/ab/$v.so $L
  timeout -k 10 200 python bench.py --config 5 --no-cpu --steps 10 --warmup 3 > gpurun_out/qab/$v.json 2> gpurun_out/qab/$v.err || { cp /tmp/base.so $L; tail -5 gpurun_out/qab/$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/qab/$v.json').read().strip().splitlines()[-1]); k=d['kernels']
print('%-8s fwd %6.2f us (%.3f)  bwd %6.2f us (%.3f)  fold %6.2f us fold2 %6.2f' % ('$v', k['qat_forward']['us'], k['qat_forward']['frac'], k['qat_backward_kernel']['us'], k['qat_backward_kernel']['frac'], k['qat_fold']['us'], k.get('qat_fold2', {}).get('us', 0)))"
done
cp /tmp/base.so $L
