"""YOLOv8 host network and the NMS oracle, on CPU.

The network cannot be pinned against ultralytics (absent offline); its
structure is pinned by ultralytics' published model summaries (parameter
counts of yolov8n/s/m at nc=80), the C3/C4/C5 channel table of SURVEY 8(a),
and the reference's backbone discovery (models/mcaq_yolo.py:351-400).
The NMS oracle is checked on hand-computed known answers."""
import numpy as np
import pytest
import torch

from mcaq_yolo_amd.yolo import DetectionModel, find_backbone_out_indices
from oracle import nms_oracle as NO

f32 = np.float32


@pytest.mark.parametrize("cfg,params,chans", [("yolov8n", 3157200, (64, 128, 256)),
                                              ("yolov8s", 11166560, (128, 256, 512)),
                                              ("yolov8m", 25902640, (192, 384, 576))])
def test_network_structure(cfg, params, chans):
    m = DetectionModel(cfg).eval()
    assert sum(p.numel() for p in m.parameters()) == params
    assert find_backbone_out_indices(m.model) == [4, 6, 9]
    shapes = {}
    hs = [m.model[i].register_forward_hook(lambda mod, a, o, k=i: shapes.__setitem__(k, tuple(o.shape)))
          for i in (4, 6, 9)]
    with torch.no_grad():
        y, raw = m(torch.rand(1, 3, 64, 96))
    for h in hs:
        h.remove()
    assert shapes[4] == (1, chans[0], 8, 12) and shapes[6] == (1, chans[1], 4, 6) and shapes[9] == (1, chans[2], 2, 3)
    assert y.shape == (1, 84, 8 * 12 + 4 * 6 + 2 * 3)
    assert [r.shape[1] for r in raw] == [144, 144, 144]
    sd = m.state_dict()
    for k in ("model.0.conv.weight", "model.2.m.0.cv1.conv.weight", "model.9.cv2.bn.running_var",
              "model.22.cv3.2.2.bias", "model.22.dfl.conv.weight"):
        assert k in sd, k


def test_backbone_discovery_fallback():
    with pytest.warns(UserWarning):
        assert find_backbone_out_indices([torch.nn.Identity()] * 12) == [4, 6, 9]


def test_detect_decode_known_answer():
    """Detect eval decode: DFL with all-equal logits -> distance 7.5 bins; box
    (cx, cy, w, h) = anchor centre, 15 strides wide."""
    m = DetectionModel("yolov8n").eval()
    det = m.model[-1]
    for seq in det.cv2:
        seq[-1].weight.data.zero_()
        seq[-1].bias.data.zero_()
    with torch.no_grad():
        y, _ = m(torch.rand(1, 3, 64, 64))
    # first anchor of P3: centre (0.5, 0.5) * 8
    assert torch.allclose(y[0, :4, 0], torch.tensor([4.0, 4.0, 120.0, 120.0]), atol=1e-4)


def test_nms_oracle_known_answers():
    # two overlapping boxes of one class (IoU 0.6806 > 0.45) + a far box; (B=1, 4+2, N=3)
    p = np.zeros((1, 6, 3), f32)
    p[0, :4, 0] = [50, 50, 20, 20]
    p[0, :4, 1] = [52, 50, 20, 20]
    p[0, :4, 2] = [200, 200, 10, 10]
    p[0, 4, :] = [0.9, 0.8, 0.3]
    out = NO.non_max_suppression(p, 0.25, 0.45)[0]
    assert out.shape == (2, 6)
    assert np.array_equal(out[:, :4], np.array([[40, 40, 60, 60], [195, 195, 205, 205]], f32))
    assert np.array_equal(out[:, 4], np.array([0.9, 0.3], f32)) and np.array_equal(out[:, 5], [0, 0])
    # second box in another class: class offset separates it
    p[0, 4, 1], p[0, 5, 1] = 0.0, 0.8
    out = NO.non_max_suppression(p, 0.25, 0.45)[0]
    assert out.shape == (3, 6) and out[1, 5] == 1
    assert NO.non_max_suppression(p, 0.25, 0.45, agnostic=True)[0].shape == (2, 6)
    # threshold is strict; max_det keeps the first kept boxes
    assert NO.non_max_suppression(p, 0.9, 0.45)[0].shape == (0, 6)
    assert NO.non_max_suppression(p, 0.25, 0.45, max_det=1)[0].shape == (1, 6)
    # IoU exactly representable ties: identical boxes -> IoU 1 suppressed; iou_thres 1.0 keeps both
    q = np.zeros((1, 5, 2), f32)
    q[0, :4, :] = np.array([[10, 10, 4, 4]], f32).T
    q[0, 4, :] = [0.5, 0.5]
    assert NO.non_max_suppression(q, 0.1, 0.45)[0].shape == (1, 6)
    assert NO.non_max_suppression(q, 0.1, 1.0)[0].shape == (2, 6)


def test_checkpoint_loading_checks_keys(tmp_path):
    """a bare DetectionModel state_dict is remapped, a checkpoint
    missing detector weights raises instead of running on random weights."""
    from mcaq_yolo_amd.yolo import MCAQYOLO
    torch.manual_seed(0)
    src = MCAQYOLO("yolov8n", device="cpu")
    bare = {k[len("model."):]: v for k, v in src.state_dict().items() if k.startswith("model.")}
    dst = MCAQYOLO("yolov8n", device="cpu")
    dst.load_checkpoint(bare)
    k = "model.model.0.conv.weight"
    assert torch.equal(dst.state_dict()[k], src.state_dict()[k])
    partial = {kk: v for kk, v in src.state_dict().items() if not kk.startswith("model.model.22")}
    with pytest.raises(RuntimeError, match="unloaded"):
        dst.load_checkpoint(partial)


def test_conv_bn_fuse_matches_unfused():
    """DetectionModel.fuse() (Conv + eval BatchNorm folded, ultralytics'
    inference default) gives the same detections head output to fp32
    rounding, and leaves no BatchNorm in the network."""
    import torch
    from mcaq_yolo_amd.yolo import DetectionModel
    torch.manual_seed(0)
    m = DetectionModel("yolov8n").eval()
    for mod in m.modules():                    # non-trivial BN statistics
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.5, 0.5)
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.2, 0.2)
    x = torch.rand(1, 3, 64, 64)
    with torch.no_grad():
        y0 = m(x)[0].clone()
        m.fuse()
        y1 = m(x)[0]
    assert not any(isinstance(mod, torch.nn.BatchNorm2d) for mod in m.modules())
    torch.testing.assert_close(y1, y0, rtol=1e-4, atol=1e-3)
