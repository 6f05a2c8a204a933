"""ctypes mirror of include/mcaq_hip.h and the loader of the native library.

The product path runs ONLY through libmcaq_hip.so (built in-tree by
__graft_entry__.build() / tools/build.py).  There is no CPU fallback: when the
library is missing or no GPU is visible, `lib()` raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libmcaq_hip.so")
ABI_VERSION = 28
DTYPE_F32, DTYPE_F16, DTYPE_BF16 = 0, 1, 2   # MCAQ_DTYPE_*
MAX_SEGMENTS = 9   # MCAQ_MAX_SEGMENTS: segments (hook scale x batch) per launch

P = ctypes.c_void_p
I = ctypes.c_int
Fl = ctypes.c_float


class StatsScale(ctypes.Structure):
    _fields_ = [("x", P), ("gray", P), ("absmean", P), ("pmin", P), ("pmax", P),
                ("B", I), ("C", I), ("H", I), ("W", I), ("Hc", I), ("Wc", I), ("unit_begin", I), ("dtype", I)]


class FinalizeScale(ctypes.Structure):
    _fields_ = [("pmin", P), ("pmax", P), ("min_in", P), ("max_in", P), ("min_out", P), ("max_out", P),
                ("C", I), ("nunits", I), ("min_stride", I), ("block_begin", I), ("per_tensor", I),
                ("neg_min", I)]


class MorphScale(ctypes.Structure):
    _fields_ = [("gray", P), ("absmean", P), ("cmlp", P), ("mapper", P), ("smask", P),
                ("c_in", P), ("bits_in", P), ("phi_out", P), ("cmlp_out", P), ("c_out", P),
                ("bits_out", P), ("m_out", P), ("mt_out", P), ("edge_out", P), ("bin_out", P), ("gscratch", P), ("tile_tmp", P),
                ("B", I), ("H", I), ("W", I), ("Hc", I), ("Wc", I), ("tile", I), ("ht", I), ("wt", I),
                ("batch_offset", I), ("batch_total", I), ("flags", I), ("hyst_iters", I),
                ("temperature", Fl), ("min_bits", Fl), ("max_bits", Fl), ("block_begin", I),
                ("softmax_threads", I), ("pwork", P)]


class QuantScale(ctypes.Structure):
    _fields_ = [("x", P), ("y", P), ("bits", P), ("m", P), ("mt", P), ("xmin", P), ("xmax", P),
                ("B", I), ("C", I), ("H", I), ("W", I), ("ht", I), ("wt", I),
                ("bits_lo", I), ("nbits", I), ("compat_tile_h", I), ("compat_tile_w", I), ("unit_begin", I),
                ("stats_cover_x", I), ("neg_min", I), ("dtype", I), ("ydtype", I)]


class QatScale(ctypes.Structure):
    _fields_ = [("x", P), ("g", P), ("y", P), ("gx", P), ("gm", P), ("gb", P), ("work", P),
                ("bits", P), ("m", P), ("xmin", P), ("xmax", P),
                ("B", I), ("C", I), ("H", I), ("W", I), ("ht", I), ("wt", I),
                ("unit_begin", I), ("block_begin", I), ("arrive", P)]


class MapperParams(ctypes.Structure):
    """mcaq_mapper_params: the train-mode mapper's tensors (torch layouts)."""
    _fields_ = [(n, P) for n in ("w1", "b1", "g1", "be1", "rm1", "rv1", "nbt1", "w2", "b2", "g2", "be2", "rm2",
                                 "rv2", "nbt2", "w3", "b3", "g3", "be3", "rm3", "rv3", "nbt3", "w4", "b4")]


class CmlpParams(ctypes.Structure):
    _fields_ = [(n, P) for n in ("w1", "b1", "g1", "be1", "w2", "b2", "g2", "be2", "w3", "b3")]


MCAQ_PACK_MAXSEG = 24


class PackSeg(ctypes.Structure):
    """mcaq_pack_seg."""
    _fields_ = [("src", P), ("n", I), ("k", I), ("mode", I), ("dst", I)]


class SmaskParams(ctypes.Structure):
    _fields_ = [(n, P) for n in ("w1", "b1", "w2", "b2")]


MCAQ_TRAIN_MAXSEG = 3
MAPPER_SYNC_STATUS_WORD = 32    # uint32 index of the fused mapper sync buffer's status word
ADAMW_SYNC_STATUS_WORD = 1      # ... and of the one-launch ClipAdamW's


class MapperSeg(ctypes.Structure):
    """mcaq_mapper_seg."""
    _fields_ = [("c", P), ("bits", P), ("work", P), ("gbits", P), ("gc", P), ("gpart", P), ("n", I)]


class HeadSeg(ctypes.Structure):
    """mcaq_head_seg."""
    _fields_ = [("phi", P), ("craw", P), ("gC", P), ("gcraw", P), ("gpart", P), ("B", I), ("ht", I), ("wt", I)]


class SmaskSeg(ctypes.Structure):
    """mcaq_smask_seg."""
    _fields_ = [("P", SmaskParams), ("bits", P), ("absmean", P), ("gm", P), ("gbits", P), ("gpart", P),
                ("B", I), ("H", I), ("W", I), ("ht", I), ("wt", I), ("accumulate", I)]


class BitBudget(ctypes.Structure):
    """mcaq_bit_budget."""
    _fields_ = [("avg", P), ("g_avg", P), ("g_loss", P), ("target", Fl), ("nscales", I)]


class QatSmaskSeg(ctypes.Structure):
    """mcaq_qat_smask_seg."""
    _fields_ = [("P", SmaskParams), ("bits", P), ("absmean", P), ("qat_work", P), ("gbits", P), ("gpart", P),
                ("B", I), ("C", I), ("H", I), ("W", I), ("ht", I), ("wt", I)]


class ReduceSeg(ctypes.Structure):
    """mcaq_reduce_seg."""
    _fields_ = [("part", P), ("out", P), ("nparts", I), ("stride", I), ("count", I), ("accumulate", I),
                ("scale", Fl)]


MCAQ_OPT_MAXSEG, MCAQ_OPT_MAXGROUPS = 64, 4


class AdamwSeg(ctypes.Structure):
    """mcaq_adamw_seg."""
    _fields_ = [("param", P), ("grad", P), ("exp_avg", P), ("exp_avg_sq", P), ("n", I), ("project_abs", I),
                ("group", I), ("step_idx", I)]


class AdamwGroup(ctypes.Structure):
    """mcaq_adamw_group."""
    _fields_ = [(k, ctypes.c_double) for k in ("lr", "weight_decay", "beta1", "beta2", "eps")]


class EmaSeg(ctypes.Structure):
    """mcaq_ema_seg."""
    _fields_ = [("batch_min", P), ("batch_max", P), ("running_min", P), ("running_max", P), ("copy_min", P),
                ("copy_max", P), ("num_batches", P), ("C", I), ("first", I), ("momentum", ctypes.c_double)]


MCAQ_DP_MAXSEG = 16


class DpSeg(ctypes.Structure):
    """mcaq_dp_seg."""
    _fields_ = [("out", P), ("off", I), ("n", I), ("mode", I)]


# morph stage flags (mcaq_morph.h)
F_PHI, F_CMLP, F_MAPPER, F_SOFTMASK = 1, 2, 4, 8
F_CONT, F_HAS_T, F_NORM_C, F_MAP_LINEAR = 16, 32, 64, 128
F_BIN_OTSU, F_NO_EULER, F_CANNY_LEGACY = 256, 512, 1024
F_TILES_IMAGE = 2048   # force the per-image pass B
F_IMAGE_BATCH = 4096   # each image as its own batch of one (the reference's batch-1 calls)

EXPORTS = ("mcaq_abi_version", "mcaq_launch_spatial_quantization", "mcaq_stats", "mcaq_stats_units",
           "mcaq_finalize", "mcaq_morph", "mcaq_morph_finalize", "mcaq_morph_scratch_bytes", "mcaq_morph_scratch_bytes_global", "mcaq_morph_work_bytes",
           "mcaq_quant",
           "mcaq_qat_forward", "mcaq_qat_backward", "mcaq_qat_work_floats", "mcaq_ema_stats",
           "mcaq_nms", "mcaq_nms_work_floats", "mcaq_time_next_launch", "mcaq_time_launch",
           "mcaq_morph_pass",
           "mcaq_mapper_work_floats", "mcaq_mapper_train_forward", "mcaq_mapper_gpart_floats",
           "mcaq_mapper_train_backward", "mcaq_head_gpart_floats", "mcaq_head_train_backward",
           "mcaq_smask_gpart_floats", "mcaq_smask_train_backward", "mcaq_ema_stats_ex", "mcaq_pack",
           "mcaq_mapper_train_forward_stage", "mcaq_mapper_train_backward_stage", "mcaq_mapper_train_reduce",
           "mcaq_mapper_train_grad_reduce", "mcaq_mapper_running_update", "mcaq_head_train_grad_reduce",
           "mcaq_mapper_train_forward_multi", "mcaq_mapper_train_backward_multi", "mcaq_head_train_backward_multi",
           "mcaq_smask_train_backward_multi", "mcaq_train_reduce_multi", "mcaq_ema_stats_multi",
           "mcaq_mapper_train_forward_stage_multi", "mcaq_mapper_train_backward_stage_multi", "mcaq_clip_adamw", "mcaq_clip_adamw_work_floats",
           "mcaq_clip_adamw_sync_bytes", "mcaq_clip_adamw_fused", "mcaq_head_sync_bytes",
           "mcaq_head_train_backward_fused",
           "mcaq_bit_budget_forward", "mcaq_qat_smask_backward_multi", "mcaq_qat_forward_budget",
           "mcaq_ema_stats_multi_running", "mcaq_head_train_backward_multi_ride",
           "mcaq_stats_pack", "mcaq_morph_ema", "mcaq_mapper_train_backward_multi_ride", "mcaq_dp_unpack",
           "mcaq_mapper_sync_bytes", "mcaq_mapper_fused_max_wg", "mcaq_mapper_train_forward_fused",
           "mcaq_mapper_train_backward_fused")

_LIB = None


class NativeLibraryMissing(RuntimeError):
    pass


def _declare(lib):
    lib.mcaq_abi_version.restype = I
    lib.mcaq_launch_spatial_quantization.restype = I
    lib.mcaq_launch_spatial_quantization.argtypes = [P, P, P, P, P, P] + [I] * 8 + [P]
    for n, st in (("mcaq_stats", StatsScale), ("mcaq_finalize", FinalizeScale),
                  ("mcaq_morph", MorphScale), ("mcaq_quant", QuantScale),
                  ("mcaq_qat_forward", QatScale), ("mcaq_qat_backward", QatScale)):
        f = getattr(lib, n)
        f.restype = I
        f.argtypes = [ctypes.POINTER(st), I, P]
    lib.mcaq_morph_finalize.restype = I
    lib.mcaq_morph_finalize.argtypes = [ctypes.POINTER(MorphScale), I, ctypes.POINTER(FinalizeScale), I, P]
    lib.mcaq_morph_pass.restype = I
    lib.mcaq_morph_pass.argtypes = [ctypes.POINTER(MorphScale), I, ctypes.POINTER(FinalizeScale), I, I, P]
    lib.mcaq_stats_units.restype = I
    lib.mcaq_stats_units.argtypes = [I, I, I, I]
    lib.mcaq_morph_scratch_bytes.restype = ctypes.c_size_t
    lib.mcaq_morph_scratch_bytes.argtypes = [I, I, I, I, I]
    lib.mcaq_morph_scratch_bytes_global.restype = ctypes.c_size_t
    lib.mcaq_morph_scratch_bytes_global.argtypes = [I, I, I]
    lib.mcaq_morph_work_bytes.restype = ctypes.c_size_t
    lib.mcaq_morph_work_bytes.argtypes = [I, I, I, I]
    lib.mcaq_qat_work_floats.restype = ctypes.c_size_t
    lib.mcaq_qat_work_floats.argtypes = [I, I, I, I]
    lib.mcaq_ema_stats.restype = I
    lib.mcaq_ema_stats.argtypes = [P, P, P, P, I, ctypes.c_double, I, P]
    lib.mcaq_nms.restype = I
    lib.mcaq_nms.argtypes = [P, I, I, I, I, Fl, ctypes.c_double, I, I, Fl, I, P, P, P, P]
    lib.mcaq_nms_work_floats.restype = ctypes.c_size_t
    lib.mcaq_nms_work_floats.argtypes = [I, I, I]
    lib.mcaq_time_next_launch.restype = I
    lib.mcaq_time_next_launch.argtypes = [P, P]
    lib.mcaq_time_launch.restype = I
    lib.mcaq_time_launch.argtypes = [I, P, P]
    SZ = ctypes.c_size_t
    for n in ("mcaq_mapper_work_floats", "mcaq_mapper_gpart_floats", "mcaq_head_gpart_floats",
              "mcaq_smask_gpart_floats"):
        getattr(lib, n).restype = SZ
        getattr(lib, n).argtypes = [I]
    lib.mcaq_mapper_train_forward.restype = I
    lib.mcaq_mapper_train_forward.argtypes = [ctypes.POINTER(MapperParams), P, I, Fl, Fl, Fl, Fl, I, I, P, P, P, P]
    lib.mcaq_mapper_train_backward.restype = I
    lib.mcaq_mapper_train_backward.argtypes = [ctypes.POINTER(MapperParams), P, I, P, Fl, Fl, Fl, P, P, P, P, I, P, P]
    lib.mcaq_mapper_train_forward_stage.restype = I
    lib.mcaq_mapper_train_forward_stage.argtypes = [ctypes.POINTER(MapperParams), P, I, Fl, Fl, Fl, Fl, I, I, P, P, I, P,
                                                    I, P]
    lib.mcaq_mapper_train_backward_stage.restype = I
    lib.mcaq_mapper_train_backward_stage.argtypes = [ctypes.POINTER(MapperParams), P, I, P, Fl, Fl, Fl, P, P, P, I, P,
                                                     P, I, P]
    lib.mcaq_mapper_train_reduce.restype = I
    lib.mcaq_mapper_train_reduce.argtypes = [P, I, I, I, P, P]
    lib.mcaq_mapper_train_grad_reduce.restype = I
    lib.mcaq_mapper_train_grad_reduce.argtypes = [I, P, P, I, P]
    lib.mcaq_mapper_running_update.restype = I
    lib.mcaq_mapper_running_update.argtypes = [ctypes.POINTER(MapperParams), ctypes.POINTER(P), ctypes.POINTER(I), I,
                                               Fl, P]
    lib.mcaq_head_train_grad_reduce.restype = I
    lib.mcaq_head_train_grad_reduce.argtypes = [I, P, P, I, P]
    lib.mcaq_mapper_train_forward_multi.restype = I
    lib.mcaq_mapper_train_forward_multi.argtypes = [ctypes.POINTER(MapperParams), ctypes.POINTER(MapperSeg), I, Fl, Fl,
                                                    Fl, Fl, I, I, P]
    lib.mcaq_mapper_train_forward_stage_multi.restype = I
    lib.mcaq_mapper_train_forward_stage_multi.argtypes = [ctypes.POINTER(MapperParams), ctypes.POINTER(MapperSeg), I,
                                                          Fl, Fl, Fl, Fl, I, I, I, ctypes.POINTER(P), I, P]
    lib.mcaq_mapper_train_backward_stage_multi.restype = I
    lib.mcaq_mapper_train_backward_stage_multi.argtypes = [ctypes.POINTER(MapperParams), ctypes.POINTER(MapperSeg),
                                                           I, Fl, Fl, Fl, I, ctypes.POINTER(P), ctypes.POINTER(P), I,
                                                           P]
    lib.mcaq_mapper_train_backward_multi.restype = I
    lib.mcaq_mapper_train_backward_multi.argtypes = [ctypes.POINTER(MapperParams), ctypes.POINTER(MapperSeg), I, Fl,
                                                     Fl, Fl, P]
    lib.mcaq_mapper_train_backward_multi_ride.restype = I
    lib.mcaq_mapper_train_backward_multi_ride.argtypes = [ctypes.POINTER(MapperParams), ctypes.POINTER(MapperSeg), I,
                                                          Fl, Fl, Fl, ctypes.POINTER(ReduceSeg), I, P]
    lib.mcaq_mapper_sync_bytes.restype = SZ
    lib.mcaq_mapper_sync_bytes.argtypes = [I]
    lib.mcaq_mapper_fused_max_wg.restype = I
    lib.mcaq_mapper_fused_max_wg.argtypes = []
    lib.mcaq_mapper_train_forward_fused.restype = I
    lib.mcaq_mapper_train_forward_fused.argtypes = [ctypes.POINTER(MapperParams), ctypes.POINTER(MapperSeg), I, Fl, Fl,
                                                    Fl, Fl, I, I, P, SZ, P]
    lib.mcaq_mapper_train_backward_fused.restype = I
    lib.mcaq_mapper_train_backward_fused.argtypes = [ctypes.POINTER(MapperParams), ctypes.POINTER(MapperSeg), I, Fl,
                                                     Fl, Fl, ctypes.POINTER(ReduceSeg), I, P, SZ, P]
    lib.mcaq_head_sync_bytes.restype = SZ
    lib.mcaq_head_sync_bytes.argtypes = [I]
    lib.mcaq_head_train_backward_fused.restype = I
    lib.mcaq_head_train_backward_fused.argtypes = [ctypes.POINTER(CmlpParams), ctypes.POINTER(HeadSeg), I,
                                                   ctypes.POINTER(ReduceSeg), I, P, I, Fl, P, SZ, P]
    lib.mcaq_head_train_backward_multi_ride.restype = I
    lib.mcaq_head_train_backward_multi_ride.argtypes = [ctypes.POINTER(CmlpParams), ctypes.POINTER(HeadSeg), I,
                                                        ctypes.POINTER(ReduceSeg), I, P]
    lib.mcaq_head_train_backward_multi.restype = I
    lib.mcaq_head_train_backward_multi.argtypes = [ctypes.POINTER(CmlpParams), ctypes.POINTER(HeadSeg), I, P]
    lib.mcaq_smask_train_backward_multi.restype = I
    lib.mcaq_smask_train_backward_multi.argtypes = [ctypes.POINTER(SmaskSeg), I, P]
    lib.mcaq_ema_stats_multi.restype = I
    lib.mcaq_ema_stats_multi.argtypes = [ctypes.POINTER(EmaSeg), I, P]
    lib.mcaq_train_reduce_multi.restype = I
    lib.mcaq_train_reduce_multi.argtypes = [ctypes.POINTER(ReduceSeg), I, I, P]
    lib.mcaq_head_train_backward.restype = I
    lib.mcaq_head_train_backward.argtypes = [ctypes.POINTER(CmlpParams), P, P, P, I, I, I, P, P, P, I, P]
    lib.mcaq_ema_stats_ex.restype = I
    lib.mcaq_ema_stats_ex.argtypes = [P, P, P, P, I, ctypes.c_double, I, P, P, P, P]
    lib.mcaq_morph_ema.restype = I
    lib.mcaq_morph_ema.argtypes = [ctypes.POINTER(MorphScale), I, ctypes.POINTER(EmaSeg), I,
                                   ctypes.POINTER(MapperParams), ctypes.POINTER(P), ctypes.POINTER(I), I, Fl, P]
    lib.mcaq_stats_pack.restype = I
    lib.mcaq_stats_pack.argtypes = [ctypes.POINTER(StatsScale), I, ctypes.POINTER(PackSeg), I, P, I, P]
    lib.mcaq_pack.restype = I
    lib.mcaq_pack.argtypes = [ctypes.POINTER(PackSeg), I, P, I, P]
    lib.mcaq_qat_forward_budget.restype = I
    lib.mcaq_qat_forward_budget.argtypes = [ctypes.POINTER(QatScale), I, ctypes.POINTER(P), ctypes.POINTER(I), I, Fl,
                                            P, P, P]
    lib.mcaq_ema_stats_multi_running.restype = I
    lib.mcaq_ema_stats_multi_running.argtypes = [ctypes.POINTER(EmaSeg), I, ctypes.POINTER(MapperParams),
                                                 ctypes.POINTER(P), ctypes.POINTER(I), I, Fl, P]
    lib.mcaq_bit_budget_forward.restype = I
    lib.mcaq_bit_budget_forward.argtypes = [ctypes.POINTER(P), ctypes.POINTER(I), I, Fl, P, P, P]
    lib.mcaq_qat_smask_backward_multi.restype = I
    lib.mcaq_qat_smask_backward_multi.argtypes = [ctypes.POINTER(QatSmaskSeg), I, ctypes.POINTER(BitBudget), P]
    lib.mcaq_clip_adamw.restype = I
    lib.mcaq_clip_adamw.argtypes = [ctypes.POINTER(AdamwSeg), I, P, I, P, Fl, P, P, P]
    lib.mcaq_clip_adamw_work_floats.restype = ctypes.c_size_t
    lib.mcaq_clip_adamw_work_floats.argtypes = [I]
    lib.mcaq_clip_adamw_sync_bytes.restype = ctypes.c_size_t
    lib.mcaq_clip_adamw_sync_bytes.argtypes = [I, I]
    lib.mcaq_clip_adamw_fused.restype = I
    lib.mcaq_clip_adamw_fused.argtypes = [ctypes.POINTER(AdamwSeg), I, P, I, P, Fl, P, P, ctypes.c_size_t, P]
    lib.mcaq_dp_unpack.restype = I
    lib.mcaq_dp_unpack.argtypes = [P, I, I, ctypes.POINTER(DpSeg), I, P]
    lib.mcaq_smask_train_backward.restype = I
    lib.mcaq_smask_train_backward.argtypes = [ctypes.POINTER(SmaskParams), P, P, P, I, I, I, I, I, P, I, P, P, P]
    return lib


def load_library(path=LIB_PATH):
    """dlopen the native library (no GPU needed: it only registers kernels)."""
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            "libmcaq_hip.so not built (%s); run `python -c 'import __graft_entry__ as g; g.build()'`" % path)
    import torch  # noqa: F401  (loads torch's libamdhip64 first: one HIP runtime per process)
    lib = _declare(ctypes.CDLL(path))
    v = lib.mcaq_abi_version()
    if v != ABI_VERSION:
        raise NativeLibraryMissing("libmcaq_hip.so ABI %d != expected %d (rebuild)" % (v, ABI_VERSION))
    return lib


def lib():
    global _LIB
    if _LIB is None:
        _LIB = load_library()
    return _LIB


def check(err, what):
    if err != 0:
        raise RuntimeError("%s failed: hipError %d" % (what, err))
