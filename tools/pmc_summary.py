"""Summarise the PMC passes of tools/pmc_traffic.sh: average HBM-side bytes per
launch of each kernel (FETCH_SIZE doubled for the gfx950 16-byte-read tally,
MI355X_MICROARCH.md "HBM"), and per hook-path step."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(root, counter):
    files = glob.glob(os.path.join(root, "pmc_%s" % counter, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            per[name].append(float(r["Counter_Value"]))
    return per


def short(name):
    if "mcaq_qat_kernel<true" in name:
        return "mcaq_qat_kernel<bwd>"
    if "mcaq_qat_kernel<false" in name:
        return "mcaq_qat_kernel<fwd>"
    for k in ("mcaq_stats_kernel", "mcaq_morph_kernel", "mcaq_tiles_kernel", "mcaq_quant_tile_kernel",
              "mcaq_quant_kernel", "mcaq_finalize", "mcaq_tb_head_kernel", "mcaq_tb_map_kernel", "mcaq_tb_mask_kernel"):
        if k in name:
            return k
    return name[:40]


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    fetch, write = load(root, "FETCH_SIZE"), load(root, "WRITE_SIZE")
    out = {"units": "bytes per launch (FETCH_SIZE kB x 1024 x 2, WRITE_SIZE kB x 1024)", "kernels": {}}
    step = 0.0
    for name in sorted(set(fetch) | set(write)):
        k = short(name)
        f = 2 * 1024 * sum(fetch.get(name, [0])) / max(len(fetch.get(name, [])), 1)
        w = 1024 * sum(write.get(name, [0])) / max(len(write.get(name, [])), 1)
        if k in out["kernels"]:          # several template instances of one kernel
            k = name[:60]
        out["kernels"][k] = {"read": round(f), "write": round(w), "total": round(f + w),
                             "launches": max(len(fetch.get(name, [])), len(write.get(name, [])))}
        if k.startswith("mcaq_"):
            step += f + w
    # per-launch sums of the hook kernels = one launch set of `batches`
    # batches (bench.py --launch-batches, the default 2 since round 5);
    # step_total is per batch, as the bench's step
    nb = int(os.environ.get("MCAQ_PMC_BATCHES", "1"))
    out["batches_per_launch"] = nb
    out["launch_total"] = round(step)
    out["step_total"] = round(step / nb)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
