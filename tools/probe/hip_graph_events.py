"""Probe: raw HIP stream capture with external timing-event record nodes
(hipEventRecordWithFlags(..., hipEventRecordExternal)) around the hook kernels."""
import ctypes, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench
from mcaq_yolo_amd.engine import HookPlan, ScaleGeom

hip = ctypes.CDLL("libamdhip64.so")
V = ctypes.c_void_p
def ck(e, what):
    if e != 0:
        raise RuntimeError("%s -> %d" % (what, e))
dev = torch.device("cuda:0")
name, B, chans, grid, mapper = bench.CONFIGS[2]
feats = [bench.synth_features(B, c, h, w, 2000 + i, dev) for i, (c, (h, w)) in enumerate(zip(chans, bench.SIZES))]
cm, mm, sm = bench.load_blobs(dev)
plan = HookPlan([ScaleGeom(B, c, h, w, grid) for c, (h, w) in zip(chans, bench.SIZES)], dev)
plan.prepare(feats, cm, mm, [sm] * 3)
st = torch.cuda.Stream()
sh = V(st.cuda_stream)
for _ in range(2):
    plan.launch(st)
torch.cuda.synchronize()
evs = []
for _ in range(4):
    e = V()
    ck(hip.hipEventCreate(ctypes.byref(e)), "hipEventCreate")
    evs.append(e)
print("has hipEventRecordWithFlags:", hasattr(hip, "hipEventRecordWithFlags"))
ck(hip.hipStreamBeginCapture(sh, 2), "begin")   # relaxed
ck(hip.hipEventRecordWithFlags(evs[0], sh, 1), "rec0")
plan.launch_stats(st)
ck(hip.hipEventRecordWithFlags(evs[1], sh, 1), "rec1")
plan.launch_morph(st)
ck(hip.hipEventRecordWithFlags(evs[2], sh, 1), "rec2")
plan.launch_quant(st)
ck(hip.hipEventRecordWithFlags(evs[3], sh, 1), "rec3")
g = V()
ck(hip.hipStreamEndCapture(sh, ctypes.byref(g)), "end")
ex = V()
ck(hip.hipGraphInstantiate(ctypes.byref(ex), g, None, None, 0), "inst")
f = ctypes.c_float()
for it in range(5):
    ck(hip.hipGraphLaunch(ex, sh), "launch")
    ck(hip.hipStreamSynchronize(sh), "sync")
    d = []
    for a, b in ((0, 1), (1, 2), (2, 3), (0, 3)):
        ck(hip.hipEventElapsedTime(ctypes.byref(f), evs[a], evs[b]), "elapsed")
        d.append(f.value * 1e3)
    print("replay %d: stats %.1f  morph %.1f  quant %.1f  total %.1f us" % (it, *d))
# eager reference with torch events
e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
with torch.cuda.stream(st):
    e[0].record(st); plan.launch_stats(st); e[1].record(st); plan.launch_morph(st); e[2].record(st); plan.launch_quant(st); e[3].record(st)
torch.cuda.synchronize()
print("eager: stats %.1f morph %.1f quant %.1f" % tuple(e[i].elapsed_time(e[i + 1]) * 1e3 for i in range(3)))
