#!/bin/bash
# QAT step (bench --config 5): concurrent vs sequential scales, HIP graph vs
# eager, HIP graph packet capture on/off.  Tag $1.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r04_qat_ab}
mkdir -p $R/gpurun_out/$T
cd $R
for r in 1 2; do
  for sc in ${SCALES:-multi concurrent sequential}; do
    for pc in ${PCS:-default}; do
      if [ $pc = default ]; then unset DEBUG_CLR_GRAPH_PACKET_CAPTURE; else export DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc; fi
      for mode in graph eager; do
        ex=""; [ $mode = eager ] && ex="--eager"
        timeout -k 10 120 python bench.py --config 5 --no-cpu --steps 100 --qat-scales $sc $ex > gpurun_out/$T/q_${sc}_${pc}_${mode}_$r.json 2> gpurun_out/$T/q_${sc}_${pc}_${mode}_$r.err || { tail -5 gpurun_out/$T/q_${sc}_${pc}_${mode}_$r.err; exit 1; }
        python -c "
import json; d=json.load(open('gpurun_out/$T/q_${sc}_${pc}_${mode}_$r.json')); print('$sc pc=$pc $mode $r', round(d['value']), round(d['ms_per_step']*1e3,1))"
      done
    done
  done
done
unset DEBUG_CLR_GRAPH_PACKET_CAPTURE
