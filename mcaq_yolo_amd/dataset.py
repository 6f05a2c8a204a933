"""Curriculum scoring of a whole dataset: the tensor path
of the reference's `compute_dataset_complexity` (mcaq_yolo/utils/dataset.py:
276-401; Algorithm 3 line 1, SortByComplexity) on the morph kernel.

The reference scores one image at a time (its collate returns one item,
:322-335): per image `x.unsqueeze(0).float()`, `/ 255` when `x.max() > 1.5`,
`analyzer.score_image(x).mean().item()` - one launch chain and one
device-to-host sync per image (:336-354).  Here consecutive images of one
shape go through the phi kernel `batch_size` at a time, each scored exactly
as its own batch-1 call would be (morph flag F_IMAGE_BATCH: the ATen
reductions whose order follows a tile's position in the batch see every
image alone), the scores stay on the device, and the host syncs once at the
end before the `.npy` save (:387-392).  So the returned array equals the
reference's for any batch_size.

The reference's fallback without an analyzer (edge density by cv2.Canny on a
cv2 RGB->gray conversion, :356-381) needs OpenCV, which this image lacks: it
raises NotImplementedError, as the analyzer's cv2 metric backend does.
"""
from typing import Optional

import numpy as np
import torch


def _item_image(item):
    """The image of one dataset item as the reference's loop takes it
    (dataset.py:337-341): item["img"] for dicts, item[0] otherwise."""
    if isinstance(item, dict):
        return item["img"]
    if isinstance(item, (tuple, list)):
        return item[0]
    return item


def _resolve_analyzer(model):
    """dataset.py:301-308: model.complexity_analyzer, or the analyzer itself."""
    if model is None:
        return None
    an = getattr(model, "complexity_analyzer", None)
    if an is None and hasattr(model, "score_image"):
        an = model
    if an is not None and not hasattr(an, "score_image"):
        an = None
    return an


def _edge_density_unavailable():
    raise NotImplementedError("compute_dataset_complexity without a complexity analyzer (or on non-tensor images) "
                              "is the reference's edge-density fallback (cv2.cvtColor + cv2.Canny, "
                              "utils/dataset.py:356-381); OpenCV is not available on this path")


def score_batch(analyzer, imgs):
    """Scores of a (B, C, H, W) batch of dataset images, each exactly as the
    reference's per-image call: float, / 255 when that image's max > 1.5,
    score_image as a batch of one (analyzer.score_image(image_batch=True)).
    Returns a (B,) fp32 tensor on the images' device; no host sync."""
    x = imgs.float()
    big = x.amax(dim=(1, 2, 3)) > 1.5                 # dataset.py:347-348, per image
    # a true IEEE division, as the reference's CPU x / 255.0: a divisor held
    # as a device tensor (ATen's CUDA kernel turns a host-scalar divisor into
    # a multiplication by its reciprocal, which rounds differently)
    x = torch.where(big.view(-1, 1, 1, 1), x / torch.full((), 255.0, device=x.device), x)
    with torch.no_grad():
        return analyzer.score_image(x, image_batch=True)


def compute_dataset_complexity(dataset, model: Optional[torch.nn.Module] = None, batch_size: int = 32,
                               device: str = "cuda", save_path: Optional[str] = None,
                               backend: Optional[str] = None, verbose: bool = True) -> np.ndarray:
    """utils/dataset.py:276-401 (same arguments and return: one float32 score
    per dataset item, in dataset order, saved to `save_path` with np.save).
    batch_size: images per launch (the reference ignores it and scores one
    image at a time; the scores do not depend on it).  backend: the
    analyzer's metric backend for scoring (only 'gpu', the tensor path,
    exists here)."""
    an = _resolve_analyzer(model)
    if an is None:
        _edge_density_unavailable()
    prev = getattr(an, "metric_backend", None)
    if backend is not None and backend != prev:
        if backend != "gpu":
            raise NotImplementedError("metric_backend=%r: only the tensor ('gpu') backend exists on this path"
                                      % backend)
        an.metric_backend = backend
    dev = torch.device(device)
    bs = max(1, int(batch_size))
    n = len(dataset)
    if verbose:
        print("Computing complexity for %d samples..." % n)
    scores = torch.empty(n, dtype=torch.float32, device=dev)
    pend, pend_idx = [], []

    def flush():
        if not pend:
            return
        xb = torch.stack(pend)
        if dev.type == "cuda":
            xb = xb.pin_memory().to(dev, non_blocking=True) if not xb.is_cuda else xb.to(dev)
        else:
            xb = xb.to(dev)
        s = score_batch(an, xb)
        scores[pend_idx[0]:pend_idx[0] + len(pend)] = s
        pend.clear()
        pend_idx.clear()

    try:
        for i in range(n):
            img = _item_image(dataset[i])
            if not isinstance(img, torch.Tensor):
                _edge_density_unavailable()
            if img.dim() == 4 and img.shape[0] == 1:
                img = img[0]
            if img.dim() != 3:
                raise ValueError("dataset item %d: expected a (C, H, W) image, got %s" % (i, tuple(img.shape)))
            if pend and (img.shape != pend[0].shape or img.dtype != pend[0].dtype or len(pend) == bs):
                flush()
            pend.append(img)
            pend_idx.append(i)
        flush()
        out = scores.cpu().numpy().astype(np.float32)     # the one device-to-host sync
    finally:
        if backend is not None and prev is not None:
            an.metric_backend = prev
    if save_path is not None:
        np.save(str(save_path), out)
        if verbose:
            print("Saved complexity scores to %s" % save_path)
    if verbose and out.size:
        print("Complexity statistics:")
        print("  Mean: %.4f" % out.mean())
        print("  Std : %.4f" % out.std())
        print("  Min : %.4f" % out.min())
        print("  Max : %.4f" % out.max())
    return out
