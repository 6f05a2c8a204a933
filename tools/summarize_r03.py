"""Summarise a gpurun_out/<tag> directory: bench lines and rocprofv3 kernel stats."""
import csv
import glob
import json
import sys

d = sys.argv[1]
for f in sorted(glob.glob(d + "/b*.json")):
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:     # noqa: BLE001
        print(f, "unreadable", e)
        continue
    if "kernels" not in j or "path_roofline" not in j:
        print(f, json.dumps(j)[:300])
        continue
    k = j["kernels"]
    print("%-34s %8.0f img/s step %5.1f us path %.3f | stats %.1f (seq %.1f) quant %.1f (seq %.1f) morph %.1f | lat %.3f ms enq %.1f us"
          % (f.split("/")[-1], j["value"], j["ms_per_step"] * 1e3, j["path_roofline"]["frac"],
             k["stats"]["us"], k["stats"].get("us_in_sequence", 0), k["quant"]["us"], k["quant"].get("us_in_sequence", 0),
             k["morph_finalize"]["us"], j["config"].get("latency_ms_single_batch", 0),
             j["config"].get("host_enqueue_us_per_step", 0)))
    if j.get("cpu_baseline"):
        print("   cpu_baseline", j["cpu_baseline"]["value"], j["cpu_baseline"]["cores"])
    if j.get("e2e"):
        print("   e2e", {k_: j["e2e"].get(k_) for k_ in ("value", "ms_per_step")}, j["e2e"].get("config", {}).get("mcaq_hooks_ms_per_step"))
for f in sorted(glob.glob(d + "/**/*kernel_stats.csv", recursive=True)):
    print(f)
    for r in csv.DictReader(open(f)):
        if "mcaq" in r["Name"] or float(r["Percentage"]) > 2:
            print("   %-60s n=%6s avg %8.2f us  %5.1f%%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
