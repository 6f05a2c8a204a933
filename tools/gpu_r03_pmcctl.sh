#!/bin/bash
# FETCH_SIZE calibration for 16 / 8 / 4-byte coalesced reads (tools/probe/pmc_control.hip)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03_pmcctl
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/r03_pmcctl/fetch -o run --output-format csv -- $R/tools/probe/pmc_control > $R/gpurun_out/r03_pmcctl/fetch.log 2>&1 || { tail -5 $R/gpurun_out/r03_pmcctl/fetch.log; exit 1; }
cd $R && python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/r03_pmcctl/fetch/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print("%-40s launches %d  FETCH_SIZE %.0f kB  -> %.3f x of 100663296 B" % (k[:40], len(v), sum(v) / len(v), sum(v) / len(v) * 1024 / 100663296))
PY
