"""Golden fixtures for the train-mode (QAT) analyzer and bit mapper, generated
by running the REFERENCE itself (build container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py

train_analyzer.npz  MorphologicalComplexityAnalyzer (morphology.py:939-973) in
                    train mode on seeded features: C, and after C.backward(gc)
                    the grads of every complexity_mlp parameter.
train_mapper.npz    ComplexityToBitMappingNetwork (bit_allocation.py:218-280)
                    in train mode (batch-statistics BatchNorm), return_continuous
                    at temperature 1 and 3: bits, grad of C, grads of every
                    mapping_network parameter, running stats after the update.
Weights: the committed weights.npz (reference key names).  Written as DATA.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _refload import load_reference  # noqa: E402
from make_golden import synth_features  # noqa: E402

torch.set_num_threads(8)
morph_mod, bit_mod, _ = load_reference()


def sub(W, prefix):
    return {k[len(prefix):]: torch.from_numpy(np.array(W[k])) for k in W.files if k.startswith(prefix)}


def main():
    W = np.load(os.path.join(HERE, "weights.npz"))
    # analyzer: P4-like shape, 2 images
    a = morph_mod.MorphologicalComplexityAnalyzer(grid_size=8, device="cpu")
    a.load_state_dict(sub(W, "complexity_analyzer."))
    a.train()
    x = synth_features(2, 16, 40, 40, 9100)
    c = a(x)
    g = torch.Generator().manual_seed(9101)
    gc = torch.randn(c.shape, generator=g)
    c.backward(gc)
    out = {"x": x.numpy(), "c": c.detach().numpy(), "gc": gc.numpy()}
    for n, p in a.complexity_mlp.named_parameters():
        out["grad.complexity_mlp." + n] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "train_analyzer.npz"), **out)
    print("train_analyzer", {k: v.shape for k, v in out.items()})

    # mapper: a complexity map spanning [0, 1], two temperatures
    out = {}
    for temp in (1.0, 3.0):
        m = bit_mod.ComplexityToBitMappingNetwork(min_bits=2, max_bits=8)
        m.load_state_dict(sub(W, "bit_mapper."))
        m.train()
        g = torch.Generator().manual_seed(9200 + int(temp))
        cm = torch.rand(4, 10, 10, generator=g)
        cm.view(-1)[:2] = torch.tensor([0.0, 1.0])
        cm.requires_grad_(True)
        bits = m(cm, temp, return_continuous=True)
        gb = torch.randn(bits.shape, generator=g)
        bits.backward(gb)
        t = "t%d" % int(temp)
        out[t + ".c"] = cm.detach().numpy()
        out[t + ".bits"] = bits.detach().numpy()
        out[t + ".gb"] = gb.numpy()
        out[t + ".grad_c"] = cm.grad.numpy()
        for n, p in m.mapping_network.named_parameters():
            out[t + ".grad.mapping_network." + n] = p.grad.numpy()
        for n, b in m.mapping_network.named_buffers():
            if b.dtype.is_floating_point:
                out[t + ".buf.mapping_network." + n] = b.numpy()
    np.savez_compressed(os.path.join(HERE, "train_mapper.npz"), **out)
    print("train_mapper", len(out), "arrays")


if __name__ == "__main__":
    main()
