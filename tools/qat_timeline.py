"""Timeline of one graph-replayed QAT step (bench.py --config 5) from a
rocprofv3 kernel trace: the kernels between the last two
mcaq_mapper_running_kernel (or mcaq_ema_running_kernel, mcaq_tiles_ema_kernel) dispatches (one per step, issued after the join
of the scale streams), by queue, with start offsets and durations (us)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if any(m in r["Kernel_Name"] for m in ("mapper_running_kernel", "ema_running_kernel", "tiles_ema_kernel"))]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
a, b = marks[-k - 1], marks[-k]
seg = rows[a + 1:b + 1]
t0 = int(seg[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in seg)
print("step span %.1f us, %d kernels" % ((t1 - t0) / 1e3, len(seg)))
busy = {}
for r in seg:
    q = r["Queue_Id"]
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    busy[q] = busy.get(q, 0) + e - s
    print("q%-3s %8.1f %7.1f  %s" % (q, s / 1e3, (e - s) / 1e3, r["Kernel_Name"][:90]))
print("busy per queue (us):", {q: round(v / 1e3, 1) for q, v in busy.items()})
