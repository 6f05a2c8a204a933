#!/bin/bash
# HBM traffic per launch of the QAT step's kernels (config 5, eager;
# rocprofv3 FETCH_SIZE / WRITE_SIZE in separate passes, tools/pmc_summary.py).
# Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r05_pmc5}
D=$R/gpurun_out/$T
mkdir -p $D
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d $D/pmc_$c -o run --output-format csv -- python3 $R/bench.py --config 5 --steps 4 --warmup 2 --eager --no-cpu > $D/pmc_$c.log 2>&1 || { tail -5 $D/pmc_$c.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $D > $D/pmc_summary.json || exit 1
python3 -c "
import json; d=json.load(open('$D/pmc_summary.json'))
for k, v in d['kernels'].items():
    if k.startswith('mcaq'): print('  %-34s read %8.2f MB write %7.2f MB (%d launches)' % (k, v['read']/1e6, v['write']/1e6, v['launches']))"
