"""Summarise rocprofv3 SQ counter passes (tools/gpu/pmc_sq.sh) per kernel:
mean per launch of each counter, for the hook path's kernels."""
import csv
import glob
import sys
from collections import defaultdict

KERNELS = ("stats", "band", "edge", "morph", "tiles", "quant_tile", "quant", "finalize")


def main(d):
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            k = next((x for x in KERNELS if "mcaq_%s_kernel" % x in n), None)
            if k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted({c for k in agg for c in agg[k]})
    print("%-22s" % "counter" + "".join("%14s" % k for k in KERNELS if k in agg))
    for c in names:
        print("%-22s" % c + "".join("%14.0f" % (sum(agg[k][c]) / max(len(agg[k][c]), 1)) for k in KERNELS if k in agg))


if __name__ == "__main__":
    main(sys.argv[1])
