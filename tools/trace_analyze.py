"""Analyze a rocprofv3 kernel trace of the pipelined bench: per-kernel mean
duration inside the timed steady state, concurrency histogram, and the
per-kernel 'exclusive share' of wall time."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trace/run_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))
ks = []
for r in rows:
    n = r["Kernel_Name"]
    if "mcaq" not in n:
        continue
    short = next(x for x in ("stats", "morph", "tiles", "quant", "finalize") if "mcaq_" + x in n)
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short, r.get("Stream_Id", "")))
ks.sort()
# steady state: the last kernels (the timed region), minus the drain
n = len(ks)
ks = ks[-int(sys.argv[2]) if len(sys.argv) > 2 else -200:][:-8]
t0, t1 = ks[0][0], max(e for _, e, _, _ in ks)
dur = defaultdict(list)
for s, e, k, _ in ks:
    dur[k].append((e - s) / 1e3)
print("span %.1f us, %d kernels" % ((t1 - t0) / 1e3, len(ks)))
for k, v in sorted(dur.items()):
    print("  %-8s n=%3d mean %6.1f us  min %6.1f  max %6.1f" % (k, len(v), sum(v) / len(v), min(v), max(v)))
ev = []
for s, e, k, _ in ks:
    ev.append((s, 1, k)); ev.append((e, -1, k))
ev.sort()
cur = defaultdict(int)
last = ev[0][0]
hist = defaultdict(float)
combo = defaultdict(float)
for t, d, k in ev:
    active = tuple(sorted(x for x, c in cur.items() for _ in range(c)))
    hist[len(active)] += t - last
    combo[active] += t - last
    cur[k] += d
    last = t
tot = sum(hist.values())
print("concurrency:", {k: round(v / tot, 3) for k, v in sorted(hist.items())})
for c, v in sorted(combo.items(), key=lambda x: -x[1])[:12]:
    print("  %5.1f%%  %s" % (100 * v / tot, "+".join(c) if c else "(idle)"))
# time with no HBM-streaming kernel (pass 1 / pass 2) running, and with one / two
nstream = defaultdict(float)
for c, v in combo.items():
    nstream[sum(1 for k in c if k in ("stats", "quant"))] += v
print("streaming kernels active:", {k: round(v / tot, 3) for k, v in sorted(nstream.items())})
