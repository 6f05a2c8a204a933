#!/bin/bash
# SQ counters per kernel (one pass, 8 SQ counters max)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 --pipeline 1 --eager --no-cpu > $R/gpurun_out/pmc_sq.log 2>&1 || { tail -5 $R/gpurun_out/pmc_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAVES --kernel-trace -d $R/gpurun_out/pmc_sq2 -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 --pipeline 1 --eager --no-cpu > $R/gpurun_out/pmc_sq2.log 2>&1 || { tail -5 $R/gpurun_out/pmc_sq2.log; exit 1; }
cd $R && python - <<'PY'
import csv, glob
from collections import defaultdict
for d in ("gpurun_out/pmc_sq", "gpurun_out/pmc_sq2"):
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            k = next((x for x in ("stats", "morph", "tiles", "quant") if "mcaq_%s" % x in n), None)
            if k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in agg.items():
        print(k, {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
PY
