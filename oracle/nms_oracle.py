"""TEST INFRASTRUCTURE ONLY - CPU restatement of the detection postprocess.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product path (mcaq_yolo_amd) never does.

Restates, in numpy fp32 with the reference's op order:
  * ultralytics `non_max_suppression` (ultralytics 8.4.63, pinned in
    requirements-lock.txt:13; NOT vendored under /root/reference and not
    importable here) as called by Predictor.postprocess / predict_batch
    (mcaq_yolo/inference.py:213-219, 410-417) with its defaults
    (classes=None, agnostic=False, multi_label=False, max_nms=30000,
    max_wh=7680);
  * torchvision's CPU `nms` kernel (greedy, stable score-descending order,
    IoU = inter / (area_i + area_j - inter) in fp32, `> iou_threshold` in
    double) - torchvision is absent here as well.
Parity status: UNPINNED against ultralytics/torchvision (neither is
installed and the reference holds no NMS fixtures); the GPU kernel is checked
bit-exactly against this restatement.
"""
import numpy as np

F32 = np.float32


def xywh2xyxy(b):
    """ultralytics.utils.ops.xywh2xyxy: xy -/+ wh / 2, fp32."""
    b = np.asarray(b, F32)
    wh = b[:, 2:4] / F32(2)
    return np.concatenate([b[:, :2] - wh, b[:, :2] + wh], axis=1).astype(F32)


def nms(boxes, scores, iou_thres):
    """torchvision.ops.nms CPU semantics; returns kept indices in order."""
    boxes = np.asarray(boxes, F32)
    x1, y1, x2, y2 = boxes[:, 0], boxes[:, 1], boxes[:, 2], boxes[:, 3]
    areas = (x2 - x1) * (y2 - y1)
    order = np.argsort(-np.asarray(scores, F32), kind="stable")
    sup = np.zeros(len(order), bool)
    keep = []
    for _i, i in enumerate(order):
        if sup[i]:
            continue
        keep.append(int(i))
        rest = order[_i + 1:]
        if rest.size == 0:
            break
        xx1 = np.maximum(x1[i], x1[rest])
        yy1 = np.maximum(y1[i], y1[rest])
        xx2 = np.minimum(x2[i], x2[rest])
        yy2 = np.minimum(y2[i], y2[rest])
        w = np.maximum(F32(0), xx2 - xx1)
        h = np.maximum(F32(0), yy2 - yy1)
        inter = w * h
        ovr = inter / ((areas[i] + areas[rest]) - inter)
        sup[rest[ovr.astype(np.float64) > np.float64(iou_thres)]] = True
    return np.asarray(keep, np.int64)


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, max_det=300, agnostic=False,
                        max_nms=30000, max_wh=7680):
    """prediction (B, 4+nc, N) -> list of (n, 6) [x1, y1, x2, y2, conf, cls]."""
    pred = np.asarray(prediction, F32)
    B, no, N = pred.shape
    nc = no - 4
    out = []
    for b in range(B):
        x = pred[b].T                                   # (N, 4+nc)
        cls = x[:, 4:]
        xc = cls.max(1) > F32(conf_thres)
        x = x[xc]
        if x.shape[0] == 0:
            out.append(np.zeros((0, 6), F32))
            continue
        box = xywh2xyxy(x[:, :4])
        conf = x[:, 4:].max(1)
        j = x[:, 4:].argmax(1).astype(F32)              # first maximum
        keep = conf > F32(conf_thres)
        det = np.concatenate([box, conf[:, None], j[:, None]], axis=1)[keep]
        if det.shape[0] > max_nms:
            det = det[np.argsort(-det[:, 4], kind="stable")[:max_nms]]
        c = det[:, 5:6] * F32(0 if agnostic else max_wh)
        i = nms(det[:, :4] + c, det[:, 4], iou_thres)[:max_det]
        out.append(det[i].astype(F32))
    return out
