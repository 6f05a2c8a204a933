#!/bin/bash
# Round 6: is the config-2 line's drop from 540 k (r06_base) to ~487 k img/s
# the box or the code?  The round-5 final tree (e769c41: its bench.py, Python
# package and library, tools/probe/ab/oldtree) and the current tree,
# interleaved on one box, default bench without the CPU / e2e legs.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_oldnew
mkdir -p $O
for r in 1 2 3; do
  (cd $R/tools/probe/ab/oldtree && timeout -k 10 200 python bench.py --no-cpu --no-e2e > $O/old_$r.json 2> $O/old_$r.err) || { tail -5 $O/old_$r.err; exit 1; }
  (cd $R && timeout -k 10 200 python bench.py --no-cpu --no-e2e > $O/new_$r.json 2> $O/new_$r.err) || { tail -5 $O/new_$r.err; exit 1; }
  python3 -c "
import json
for v in ('old', 'new'):
    d = json.load(open('$O/%s_$r.json' % v)); k = d['kernels']
    print(v, $r, round(d['value']), round(d['ms_per_step'] * 1e3, 1), d['path_roofline']['frac'], 'quant', k['quant']['us'], k['quant']['us_in_sequence'], 'stats', k['stats']['us'], k['stats']['us_in_sequence'], 'morph', k['morph_finalize']['us'])"
done
