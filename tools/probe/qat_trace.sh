#!/bin/bash
# rocprofv3 kernel trace of tools/probe/qat_trace.py per variant library
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=$R/mcaq_yolo_amd/lib/libmcaq_hip.so
cp $L /tmp/base.so
for v in "$@"; do
  cp $R/tools/probe/ab/$v.so $L
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/qtr/$v -o run -- python3 $R/tools/probe/qat_trace.py > $R/gpurun_out/qtr/$v.log 2>&1) || { cp /tmp/base.so $L; tail -5 $R/gpurun_out/qtr/$v.log; exit 1; }
done
cp /tmp/base.so $L
cd $R && python3 - "$@" <<'PY'
import csv, glob, sys
for v in sys.argv[1:]:
    f = glob.glob("gpurun_out/qtr/%s/**/*kernel_trace.csv" % v, recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "qat" in r["Kernel_Name"]][-60:]
    prev = None
    out = {}
    for r in rows:
        k = "fold" if "fold" in r["Kernel_Name"] else "bwd"
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        gap = (int(r["Start_Timestamp"]) - prev) / 1e3 if prev else 0
        prev = int(r["End_Timestamp"])
        out.setdefault(k, []).append((d, gap))
    for k, l in out.items():
        print(v, k, "n=%d dur avg %.2f min %.2f  gap-before avg %.2f" % (len(l), sum(a for a, _ in l) / len(l), min(a for a, _ in l), sum(b for _, b in l) / len(l)))
PY
