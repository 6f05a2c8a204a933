#!/bin/bash
# SQ counters per kernel (two passes of <= 8 SQ counters), single-batch steps
# in sequence (bench --pipeline 1 --eager).  Tag $1 -> gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-pmc_sq}
mkdir -p $R/gpurun_out/$T
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d $R/gpurun_out/$T/p1 -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 --pipeline 1 --eager --no-cpu --no-e2e > $R/gpurun_out/$T/p1.log 2>&1 || { tail -5 $R/gpurun_out/$T/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_MFMA --kernel-trace -d $R/gpurun_out/$T/p2 -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 --pipeline 1 --eager --no-cpu --no-e2e > $R/gpurun_out/$T/p2.log 2>&1 || { tail -5 $R/gpurun_out/$T/p2.log; exit 1; }
cd $R && python3 tools/pmc_sq_summary.py gpurun_out/$T | tee gpurun_out/$T/summary.txt
