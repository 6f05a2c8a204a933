"""Probe: multi-stream HIP stream capture through torch.cuda.graph on this
ROCm, in increasing complexity; prints a line after each case (a crash names
the case that broke).  Cases:
  A  fork origin -> s1, s2 (events), kernels, join
  B  side-to-side edge: s2 waits for an event recorded on s1
  C  one event recorded twice inside the capture (ring reuse)
  C1 one event re-recorded, one direction only
  C2 both directions between two side streams (the case that segfaulted at
     hipStreamEndCapture on ROCm 7.0 / torch 2.10, round 3)"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
hip = ctypes.CDLL("libamdhip64.so")
V = ctypes.c_void_p


def say(*a):
    print(*a, flush=True)


def hstream(flags=1):
    s = V()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), flags) == 0
    return s, torch.cuda.ExternalStream(s.value)


def hevent():
    e = V()
    assert hip.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0   # disable timing
    return e


x = torch.randn(1 << 20, device="cuda")
y = torch.empty_like(x)
z = torch.empty_like(x)
cap = torch.cuda.Stream()
(h1, s1), (h2, s2) = hstream(), hstream()
ef, e1, e2, ej1, ej2 = (hevent() for _ in range(5))


def run_case(name, body):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        hc = V(cap.cuda_stream)
        body(hc)
    g.replay()
    torch.cuda.synchronize()
    say("case", name, "ok", float(y.sum()), float(z.sum()))


def fork(hc):
    assert hip.hipEventRecord(ef, hc) == 0
    assert hip.hipStreamWaitEvent(h1, ef, 0) == 0
    assert hip.hipStreamWaitEvent(h2, ef, 0) == 0


def join(hc):
    assert hip.hipEventRecord(ej1, h1) == 0
    assert hip.hipEventRecord(ej2, h2) == 0
    assert hip.hipStreamWaitEvent(hc, ej1, 0) == 0
    assert hip.hipStreamWaitEvent(hc, ej2, 0) == 0


def case_a(hc):
    fork(hc)
    with torch.cuda.stream(s1):
        y.copy_(x)
    with torch.cuda.stream(s2):
        z.copy_(x)
    join(hc)


def case_b(hc):
    fork(hc)
    with torch.cuda.stream(s1):
        y.copy_(x)
    assert hip.hipEventRecord(e1, h1) == 0
    assert hip.hipStreamWaitEvent(h2, e1, 0) == 0
    with torch.cuda.stream(s2):
        z.copy_(y)
    join(hc)


def case_c(hc):
    fork(hc)
    for _ in range(2):
        with torch.cuda.stream(s1):
            y.add_(1.0)
        assert hip.hipEventRecord(e1, h1) == 0
        assert hip.hipStreamWaitEvent(h2, e1, 0) == 0
        with torch.cuda.stream(s2):
            z.copy_(y)
        assert hip.hipEventRecord(e2, h2) == 0
        assert hip.hipStreamWaitEvent(h1, e2, 0) == 0
    join(hc)


def case_c1(hc):            # one event re-recorded, one direction only
    fork(hc)
    for _ in range(2):
        with torch.cuda.stream(s1):
            y.add_(1.0)
        assert hip.hipEventRecord(e1, h1) == 0
        assert hip.hipStreamWaitEvent(h2, e1, 0) == 0
        with torch.cuda.stream(s2):
            z.copy_(y)
    join(hc)


def case_c2(hc):            # both directions, distinct events, no re-record
    fork(hc)
    with torch.cuda.stream(s1):
        y.add_(1.0)
    assert hip.hipEventRecord(e1, h1) == 0
    assert hip.hipStreamWaitEvent(h2, e1, 0) == 0
    with torch.cuda.stream(s2):
        z.copy_(y)
    assert hip.hipEventRecord(e2, h2) == 0
    assert hip.hipStreamWaitEvent(h1, e2, 0) == 0
    with torch.cuda.stream(s1):
        y.add_(1.0)
    join(hc)


say("torch", torch.__version__, "hip", torch.version.hip)
run_case("A", case_a)
run_case("B", case_b)

run_case("C1", case_c1)
run_case("C2", case_c2)
run_case("C", case_c)
say("all ok")
