#!/bin/bash
# r03: shape probe (pass-1 channel split), pass-2 variant A/B, e2e batches in flight 1/2/3
set -o pipefail
export TMPDIR=/tmp
T=r03_mix1
mkdir -p gpurun_out/$T
timeout -k 10 120 ./tools/probe/shape_probe > gpurun_out/$T/shape_probe.txt 2>&1; rc=$?; cat gpurun_out/$T/shape_probe.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r03_ab.sh $T q_cur q_s16 q_nt3 q_nt0 q_lb8 q_lb4 || exit 1
for n in 1 2 3; do
  timeout -k 10 300 python bench.py --e2e --steps 30 --warmup 3 --e2e-inflight $n > gpurun_out/$T/e2e_$n.json 2> gpurun_out/$T/e2e_$n.err || { tail -20 gpurun_out/$T/e2e_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/$T/e2e_$n.json').read().strip().splitlines()[-1]); c=d['config']; print('e2e inflight $n', d['value'], 'img/s', d['ms_per_step'], 'ms', 'net', c['network_only_ms_per_step'], 'hooks', c['mcaq_hooks_ms_per_step'], 'share', c['hook_share_of_step'], 'dets', c['detections_per_image'])"
done
