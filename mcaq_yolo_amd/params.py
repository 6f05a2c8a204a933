"""Pack reference-layout parameter tensors into the flat blobs the kernels read.

The blob layouts are the CM_* / MM_* / SM_* offsets of
mcaq_yolo_amd/csrc/mcaq_morph.h (reference parameter order), followed for the
two MLPs by the weight matrices re-laid-out as fp32 MFMA A operands
(CMQ_* / MMQ_* in mcaq_mlp_mfma.h).  Input: mappings from the reference
state_dict key suffixes (complexity_mlp.{0,1,3,4,6}.*, mapping_network.
{0,1,3,4,6,7,9}.*, net.{0,2}.*) to tensors or arrays.
"""
import numpy as np

CM_SIZE, MM_SIZE, SM_SIZE = 2881, 4865, 170
CMQ_SIZE = CM_SIZE + 512 + 2048      # + MFMA A-operand copies (mcaq_mlp_mfma.h)
MMQ_SIZE = MM_SIZE + 128 + 2048 + 2048


def _pad4(a):
    """Blobs are read as 16-byte vectors: pad to a multiple of 4 floats."""
    n = (-a.size) % 4
    return np.concatenate([a, np.zeros(n, np.float32)]) if n else a


def _f(a):
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.asarray(a, np.float32).reshape(-1)


def mfma_a_operands(Wm):
    """Weight matrix (N_out, K) -> A operands of v_mfma_f32_16x16x4_f32 for the
    transposed product D[neuron][tile]: [block][step][lane] with lane l holding
    W[16*block + (l & 15)][4*step + (l >> 4)] (K zero-padded to a multiple of 4)."""
    Wm = np.asarray(Wm, np.float32)
    n, k = Wm.shape
    kp = (k + 3) // 4 * 4
    nb = (n + 15) // 16
    Wp = np.zeros((nb * 16, kp), np.float32)
    Wp[:n, :k] = Wm
    lane = np.arange(64)
    out = np.empty((nb, kp // 4, 64), np.float32)
    for b in range(nb):
        for s in range(kp // 4):
            out[b, s] = Wp[16 * b + (lane & 15), 4 * s + (lane >> 4)]
    return out.reshape(-1)


def _np2(a):
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.asarray(a, np.float32)


def pack_complexity_mlp(sd, prefix="complexity_mlp."):
    """morphology.py:81-90: Linear(8,64) LN(64) ReLU Linear(64,32) LN(32) ReLU Linear(32,1)."""
    parts = [sd[prefix + "0.weight"], sd[prefix + "0.bias"], sd[prefix + "1.weight"], sd[prefix + "1.bias"],
             sd[prefix + "3.weight"], sd[prefix + "3.bias"], sd[prefix + "4.weight"], sd[prefix + "4.bias"],
             sd[prefix + "6.weight"], sd[prefix + "6.bias"]]
    out = np.concatenate([_f(p) for p in parts])
    if out.size != CM_SIZE:
        raise ValueError("complexity MLP must be the reference 8-64-32-1 shape (got %d params)" % out.size)
    return _pad4(np.concatenate([out, mfma_a_operands(_np2(sd[prefix + "0.weight"])),
                                 mfma_a_operands(_np2(sd[prefix + "3.weight"]))]))


def pack_mapper_mlp(sd, prefix="mapping_network."):
    """bit_allocation.py:119-136 with hidden_dims [32, 64, 32]."""
    parts = []
    for lin, bn in ((0, 1), (3, 4), (6, 7)):
        parts += [sd[prefix + "%d.weight" % lin], sd[prefix + "%d.bias" % lin]]
        parts += [sd[prefix + "%d.%s" % (bn, k)] for k in ("weight", "bias", "running_mean", "running_var")]
    parts += [sd[prefix + "9.weight"], sd[prefix + "9.bias"]]
    out = np.concatenate([_f(p) for p in parts])
    if out.size != MM_SIZE:
        raise ValueError("bit mapper must use hidden_dims [32, 64, 32] (got %d params)" % out.size)
    return _pad4(np.concatenate([out] + [mfma_a_operands(_np2(sd[prefix + "%d.weight" % i])) for i in (0, 3, 6)]))


def pack_soft_mask(sd, prefix="net."):
    """quantization.py:187-191: Conv2d(2,8,3) ReLU Conv2d(8,2,1)."""
    parts = [sd[prefix + "0.weight"], sd[prefix + "0.bias"], sd[prefix + "2.weight"], sd[prefix + "2.bias"]]
    out = np.concatenate([_f(p) for p in parts])
    if out.size != SM_SIZE:
        raise ValueError("soft mask must be the reference Conv2d(2,8,3)/Conv2d(8,2,1) net")
    return _pad4(out)


def sub(sd, prefix):
    """Select keys under `prefix` and strip it."""
    return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}
