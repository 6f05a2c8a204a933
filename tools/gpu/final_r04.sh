#!/bin/bash
# Round-4 validation of a build: full GPU tests, smoke, default bench lines
# (20 and 400 steps), config 5 and configs 3 / 4 bench lines.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r04_final}
cd $R
bash tools/gpu/check.sh $T || exit 1
for c in 5 3 4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-e2e > gpurun_out/$T/bench_config$c.json 2> gpurun_out/$T/bench_config$c.err || { tail -8 gpurun_out/$T/bench_config$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/$T/bench_config$c.json')); pr=d.get('path_roofline') or d.get('step_roofline'); print('config $c', round(d['value']), round(d['ms_per_step']*1e3,1), 'path/step', pr['frac'], 'roofline', d['roofline']['frac'], d['roofline']['us_per_launch'], d['roofline']['traffic'])"
done
