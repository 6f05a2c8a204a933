#!/bin/bash
# The N > 1 hook-path schedule (split graphs around an eager RCCL all-reduce
# per launch set, 3 sets in flight) rehearsed on one GPU with a world-1 RCCL
# group, beside the captured world-1 and the unsharded lines (2x interleaved).
set -o pipefail
O=gpurun_out/r06_eager_coll; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 200 > $O/unsharded.$r.json 2> $O/unsharded.$r.err || { tail -5 $O/unsharded.$r.err; exit 1; }
  MCAQ_BENCH_SHARDED=1 timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 200 > $O/captured.$r.json 2> $O/captured.$r.err || { tail -5 $O/captured.$r.err; exit 1; }
  MCAQ_BENCH_SHARDED=1 MCAQ_BENCH_EAGER_COLLECTIVE=1 timeout -k 10 200 python bench.py --no-cpu --no-e2e --steps 200 > $O/eager.$r.json 2> $O/eager.$r.err || { tail -5 $O/eager.$r.err; exit 1; }
done
for f in $O/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); c=d['config']; print(d['value'], d['ms_per_step'], c.get('rccl_in_graph'), c.get('host_enqueue_us_per_step'))")"; done
