"""Diagnostic: the multi-scale QAT step with and without the fused
mask/quantizer/bit-budget node (train_step.FUSED_MASK_QAT), step by step:
max relative difference of outputs, bit maps, complexity, gradients and
parameters (relative to each tensor's own max)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_concurrent_scales_gpu import _run  # noqa: E402

for steps in (1, 2, 3):
    a = _run(False, steps=steps, multi=True, fused_mq=True)
    b = _run(False, steps=steps, multi=True, fused_mq=False)
    worst = []
    for k in ("outs", "bits", "cplx", "fgrad"):
        for i, (x, y) in enumerate(zip(a[k], b[k])):
            worst.append((float((x - y).abs().max()) / max(float(y.abs().max()), 1e-30), "%s[%d]" % (k, i)))
    for k in ("grads", "params", "bufs"):
        for n in a[k]:
            x, y = a[k][n].float(), b[k][n].float()
            if x.numel():
                worst.append((float((x - y).abs().max()) / max(float(y.abs().max()), 1e-30), "%s %s" % (k, n)))
    worst.sort(reverse=True)
    print("steps", steps, flush=True)
    for r, n in worst[:12]:
        print("   %.3e  %s" % (r, n), flush=True)
