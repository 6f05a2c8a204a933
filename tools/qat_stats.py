"""Per-step kernel time of a rocprofv3 --stats CSV of `bench.py --config 5`
(steps = the calls of the per-step mapper forward kernel / 3 scales)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = max([int(r["Calls"]) for r in rows if "mapper_fwd_kernel<1>" in r["Name"]] or [3]) / 3.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
mc = sum(float(r["TotalDurationNs"]) for r in rows if "mcaq" in r["Name"])
print("steps %.0f  kernel time per step %.1f us (mcaq %.1f, other %.1f)" % (steps, tot / steps / 1e3, mc / steps / 1e3,
                                                                             (tot - mc) / steps / 1e3))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print("%8.1f us/step %5.1f/step avg %7.2f  %s" % (float(r["TotalDurationNs"]) / steps / 1e3, int(r["Calls"]) / steps,
                                                     float(r["AverageNs"]) / 1e3, r["Name"][:100]))
