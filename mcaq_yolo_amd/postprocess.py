"""Detection postprocess on the HIP path: batched NMS and the cross-rank
detection all-gather.

`non_max_suppression` mirrors the call the reference's Predictor makes
(mcaq_yolo/inference.py:213-219, 410-417 -> ultralytics
`non_max_suppression(preds, conf_thres, iou_thres, max_det)`): same argument
names and defaults, same output (a list of (n, 6) [x1, y1, x2, y2, conf, cls]
tensors per image).  The whole batch is ONE kernel launch (`mcaq_nms`, one
workgroup per image); `nms_padded` returns the fixed-shape (B, max_det, 6) +
counts form that is HIP-graph capturable and is what `gather_detections`
exchanges over RCCL.  Unlike ultralytics (in_place=True) the input tensor is
not modified.  Options the reference never passes (classes, multi_label,
labels, rotated, extra mask channels) raise NotImplementedError.
"""
import ctypes

import torch

from . import abi


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class NmsPlan:
    """Preallocated outputs for a fixed (B, no, N, max_det)."""

    def __init__(self, B, no, N, max_det, device):
        self.B, self.no, self.N, self.max_det = B, no, N, max_det
        self.out = torch.empty(B, max_det, 6, device=device)
        self.counts = torch.empty(B, device=device, dtype=torch.int32)
        self.work = torch.empty(max(1, abi.lib().mcaq_nms_work_floats(B, N, max_det)), device=device)

    def run(self, pred, conf_thres=0.25, iou_thres=0.45, agnostic=False, max_nms=30000, max_wh=7680):
        if not pred.is_cuda:
            raise RuntimeError("mcaq_nms runs on MI355X (HIP) only; got a %s tensor" % pred.device)
        if pred.dtype != torch.float32 or not pred.is_contiguous() or tuple(pred.shape) != (self.B, self.no, self.N):
            raise ValueError("prediction must be contiguous fp32 %s, got %s %s"
                             % ((self.B, self.no, self.N), tuple(pred.shape), pred.dtype))
        L = abi.lib()
        abi.check(L.mcaq_nms(ctypes.c_void_p(pred.data_ptr()), self.B, self.no, self.N, self.no - 4,
                             float(conf_thres), float(iou_thres), int(self.max_det), int(max_nms), float(max_wh),
                             1 if agnostic else 0, ctypes.c_void_p(self.out.data_ptr()),
                             ctypes.c_void_p(self.counts.data_ptr()), ctypes.c_void_p(self.work.data_ptr()),
                             _stream()), "mcaq_nms")
        return self.out, self.counts


_PLANS = {}


def nms_padded(prediction, conf_thres=0.25, iou_thres=0.45, max_det=300, agnostic=False, max_nms=30000,
               max_wh=7680):
    """(B, 4+nc, N) fp32 CUDA -> (B, max_det, 6) detections (zero rows past
    the count) and (B,) int32 counts.  Outputs are reused by the next call
    with the same shapes (clone to keep them)."""
    if isinstance(prediction, (list, tuple)):
        prediction = prediction[0]
    p = prediction.float().contiguous()
    key = (tuple(p.shape), max_det, p.device)
    plan = _PLANS.get(key)
    if plan is None:
        plan = _PLANS[key] = NmsPlan(p.shape[0], p.shape[1], p.shape[2], max_det, p.device)
    return plan.run(p, conf_thres, iou_thres, agnostic, max_nms, max_wh)


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                        multi_label=False, labels=(), max_det=300, nc=0, max_time_img=0.05, max_nms=30000,
                        max_wh=7680, in_place=True, rotated=False, end2end=False, return_idxs=False):
    """ultralytics-compatible signature; returns a list of (n, 6) tensors."""
    if classes is not None or multi_label or len(labels) or rotated or end2end or return_idxs:
        raise NotImplementedError("classes / multi_label / labels / rotated / end2end / return_idxs: "
                                  "not used by the reference's Predictor")
    if isinstance(prediction, (list, tuple)):
        prediction = prediction[0]
    if nc and prediction.shape[1] != 4 + nc:
        raise NotImplementedError("extra (mask) channels after the class scores")
    out, counts = nms_padded(prediction, conf_thres, iou_thres, max_det, agnostic, max_nms, max_wh)
    n = counts.tolist()                        # one device->host sync for the whole batch
    return [out[b, :n[b]].clone() for b in range(out.shape[0])]


def gather_detections(out, counts, group=None):
    """RCCL all-gather of every rank's padded detections (batch-sharded
    inference): (B_local, max_det, 6) + (B_local,) per rank ->
    (world * B_local, max_det, 6) + counts in rank order, one collective each."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":       # CPU rehearsal: gloo has no *_into_tensor gather
        outs = [torch.empty_like(out) for _ in range(world)]
        cnts = [torch.empty_like(counts) for _ in range(world)]
        dist.all_gather(outs, out.contiguous(), group=group)
        dist.all_gather(cnts, counts.contiguous(), group=group)
        return torch.cat(outs), torch.cat(cnts)
    g_out = torch.empty((world * out.shape[0],) + tuple(out.shape[1:]), device=out.device, dtype=out.dtype)
    g_cnt = torch.empty(world * counts.shape[0], device=counts.device, dtype=counts.dtype)
    dist.all_gather_into_tensor(g_out, out.contiguous(), group=group)
    dist.all_gather_into_tensor(g_cnt, counts.contiguous(), group=group)
    return g_out, g_cnt
