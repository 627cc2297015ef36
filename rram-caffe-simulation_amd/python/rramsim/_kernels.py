"""ctypes binding of the gfx950 kernel library (include/rram_kernels.h).

This is the Python-side view of the C-ABI boundary.  It is deliberately
thin: argument marshalling, status checking and a few host-side helpers that
turn the reference's parameters (fault probabilities, neg/zero/pos splits)
into the kernels' integer thresholds.  There is no CPU fallback anywhere in
this package: if the shared library is missing, importing it raises.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from pathlib import Path

_PKG_ROOT = Path(__file__).resolve().parents[2]          # rram-caffe-simulation_amd/
# RRAM_LIB_DIR: developer override to A/B kernel variants built into another
# in-tree directory (scripts/gpu_variants.sh); the product loads lib/.
LIB_DIR = Path(os.environ["RRAM_LIB_DIR"]) if os.environ.get("RRAM_LIB_DIR") else _PKG_ROOT / "lib"
KERNELS_SO = LIB_DIR / "librram_kernels.so"
CAFFE_SO = LIB_DIR / "librram_caffe.so"

RRAM_OK, RRAM_EINVAL, RRAM_EHIP, RRAM_ENOMEM, RRAM_EUNSUPPORTED = 0, -1, -2, -3, -4
RRAM_CELL_SINGLE, RRAM_CELL_DIFFPAIR = 0, 1
RRAM_BIAS_NONE, RRAM_BIAS_ROW, RRAM_BIAS_COL = 0, 1, 2
RRAM_POOL_MAX, RRAM_POOL_AVE = 0, 1
RRAM_MAX_SEGS = 32
TWO32 = 1 << 32


class RramError(RuntimeError):
    pass


class InjectCfg(C.Structure):
    _fields_ = [
        ("thr_fault", C.c_uint64), ("thr_neg", C.c_uint64), ("thr_zero", C.c_uint64),
        ("thr_sa1", C.c_uint64), ("stuck_scale", C.c_float), ("g_max", C.c_float),
        ("quant_levels", C.c_int32), ("var_sigma", C.c_float), ("cell_mode", C.c_int32),
        ("reserved", C.c_int32),
    ]


class InjectSeg(C.Structure):
    _fields_ = [("w_clean", C.c_void_p), ("w_out", C.c_void_p), ("n", C.c_int64),
                ("layer_id", C.c_uint32), ("reserved", C.c_uint32), ("cfg", InjectCfg)]


class FailSeg(C.Structure):
    _fields_ = [("dw", C.c_void_p), ("w", C.c_void_p), ("endurance", C.c_void_p),
                ("values", C.c_void_p), ("n", C.c_int64)]


class UpdateSeg(C.Structure):
    _fields_ = [("w", C.c_void_p), ("g", C.c_void_p), ("h", C.c_void_p), ("endurance", C.c_void_p),
                ("values", C.c_void_p), ("n", C.c_int64), ("decay", C.c_float), ("local_rate", C.c_float),
                ("thr", C.c_float), ("apply_thr", C.c_int), ("broken_count", C.c_void_p),
                ("w_flip", C.c_void_p), ("flip_groups", C.c_int), ("flip_cin", C.c_int), ("flip_cout", C.c_int),
                ("flip_taps", C.c_int)]


class ConvDesc(C.Structure):
    _fields_ = [(k, C.c_int) for k in (
        "num", "channels", "height", "width", "num_output", "kernel_h", "kernel_w", "pad_h",
        "pad_w", "stride_h", "stride_w", "dilation_h", "dilation_w", "group", "out_h", "out_w")]


# (name, restype, argtypes) for every symbol of include/rram_kernels.h
P, I, I64, U32, U64, F, SZ = C.c_void_p, C.c_int, C.c_int64, C.c_uint32, C.c_uint64, C.c_float, C.c_size_t
SIGNATURES = {
    "rram_kernels_version": (C.c_char_p, []),
    "rram_last_error": (C.c_char_p, []),
    "rram_device_synchronize": (I, []),
    "rram_release_caches": (I, []),
    "rram_scratch_generation": (U64, []),
    "rram_set_f32_engine": (I, [I]),
    "rram_get_f32_engine": (I, []),
    "rram_f32_engine_for_conv": (I, [P]),
    "rram_f32_engine_for_ip": (I, [I, I, I, SZ]),
    "rram_conv_output_octets_only": (I, [P]),
    "rram_fault_threshold": (I, [P, I64, F, F, P]),
    "rram_fault_init": (I, [P, P, I64, F, F, U64, U64, U64, U32, U32, P]),
    "rram_fail_apply": (I, [P, P, P, P, I64, F, F, P, P]),
    "rram_fail_apply_batched": (I, [P, I, F, F, P, P]),
    "rram_broken_count": (I, [P, I64, P, P]),
    "rram_inject_rng": (I, [P, P, I64, P, U64, U32, U32, P, P]),
    "rram_set_inject_grid": (I, [I]),
    "rram_inject_rng_batched": (I, [P, I, U64, U32, P, P]),
    "rram_threshold_strategy": (I, [P, I64, F, P, P]),
    "rram_stuck_zero_counts": (I, [P, P, I, I, P, P, P]),
    "rram_mc_accumulate": (I, [P, P, P, P]),
    "rram_permute_rows": (I, [P, P, I64, P, P, I, P]),
    "rram_permute_cols": (I, [P, P, I, I, P, P, I, P]),
    "rram_permute_elems": (I, [P, P, P, P, I, P]),
    "rram_sgd_update": (I, [P, P, I64, F, F, P]),
    "rram_fused_update_fail": (I, [P, P, P, P, P, I64, F, F, F, I, F, F, F, P, P]),
    "rram_fused_update_fail_batched": (I, [P, I, F, F, F, P]),
    "rram_axpy": (I, [I64, F, P, P, P]),
    "rram_axpby": (I, [I64, F, P, F, P, P]),
    "rram_scal": (I, [I64, F, P, P]),
    "rram_set": (I, [I64, F, P, P]),
    "rram_zero_pair": (I, [P, I64, P, I64, P]),
    "rram_add": (I, [I64, P, P, P, P]),
    "rram_sign": (I, [I64, P, P, P]),
    "rram_asum": (I, [I64, P, P, P]),
    "rram_absmax": (I, [I64, P, P, P]),
    "rram_dot": (I, [I64, P, P, P, P]),
    "rram_gemm_f32": (I, [I, I, I, I, I, F, P, P, F, P, P]),
    "rram_gemm_f32_ex": (I, [I, I, I, I, I, F, P, I, P, I, F, P, I, P, I, I, P, SZ, P]),
    "rram_gemv_f32": (I, [I, I, I, F, P, P, F, P, P]),
    "rram_conv_out_shape": (I, [P]),
    "rram_conv2d_fwd": (I, [P, P, P, P, P, I, P]),
    "rram_conv2d_fwd_octets": (I, [P, P, P, P, P, P, P, I, P]),
    "rram_conv_input_octets": (I, [P]),
    "rram_conv_octet_plan": (I, [P, P]),
    "rram_conv_weight_pack_bytes": (SZ, [P]),
    "rram_conv2d_fwd_cached": (I, [P, P, P, P, P, I, P, P, P, I, P]),
    "rram_conv2d_fwd_strided": (I, [P, P, P, P, P, I, P, P, C.c_int64, I, P]),
    "rram_inject_rng_batched_dev": (I, [P, I, C.c_uint64, P, P, P]),
    "rram_mc_accumulate_dev": (I, [P, P, P, C.c_int64, I, P, P, I, P]),
    "rram_pack_octets": (I, [P, P, I, I, I, I, P]),
    "rram_conv2d_bwd_workspace": (SZ, [P, I]),
    "rram_conv2d_bwd": (I, [P, P, P, P, P, P, P, P, SZ, P]),
    "rram_conv2d_bwd_ex": (I, [P, P, P, P, P, P, P, P, P, SZ, P]),
    "rram_conv2d_flip_applies": (I, [P]),
    "rram_im2col": (I, [P, I, I, I, I, I, I, I, I, I, I, I, P, P]),
    "rram_col2im": (I, [P, I, I, I, I, I, I, I, I, I, I, I, P, P]),
    "rram_ip_fwd": (I, [P, P, P, P, I, I, I, I, I, P, SZ, P]),
    "rram_ip_bwd": (I, [P, P, P, P, P, P, I, I, I, I, P]),
    "rram_ip_rows_pack_bytes": (SZ, [I, I, I, SZ, P]),
    "rram_ip_fwd_rows": (I, [P, P, P, P, P, P, I, I, I, I, I, P, SZ, P, P]),
    "rram_relu_fwd": (I, [P, P, I64, F, P]),
    "rram_relu_bwd": (I, [P, P, P, I64, F, P]),
    "rram_pool_fwd": (I, [P, P, P] + [I] * 13 + [P]),
    "rram_pool_relu_fwd": (I, [P, P, P] + [I] * 13 + [F, P]),
    "rram_pool_relu_bwd": (I, [P, P, P] + [I] * 13 + [P, F, P]),
    "rram_pool_bwd": (I, [P, P, P] + [I] * 13 + [P]),
    "rram_lrn_fwd": (I, [P, P, P, I, I, I, I, I, F, F, F, P]),
    "rram_lrn_bwd": (I, [P, P, P, P, P, I, I, I, I, I, F, F, P]),
    "rram_lrn_within_fwd": (I, [P, P, P, I, I, I, I, I, F, F, P]),
    "rram_lrn_within_bwd": (I, [P, P, P, P, I, I, I, I, I, F, F, P]),
    "rram_lrn_within_relu_bwd": (I, [P, P, P, P, I, I, I, I, I, F, F, F, P]),
    "rram_lrn_maxpool_fwd": (I, [P, P, I, I, I, I, I, I, I, I, I, I, I, I, F, F, F, P]),
    "rram_lrn_maxpool_fwd_octets": (I, [P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, F, F, F, P]),
    "rram_softmax_fwd": (I, [P, P, I, I, I, P]),
    "rram_softmax_loss_fwd": (I, [P, P, P, I, I, I, I, P]),
    "rram_softmax_loss_fwd_acc": (I, [P, P, P, I, I, I, I, P, P, P]),
    "rram_softmax_loss_bwd": (I, [P, P, P, I, I, I, I, F, P]),
    "rram_softmax_loss_fwd_bwd": (I, [P, P, P, P, I, I, I, I, F, P]),
    "rram_accuracy": (I, [P, P, P, P, P, I, I, I, I, I, P]),
    "rram_accuracy_acc": (I, [P, P, P, P, P, I, I, I, I, I, P, P, P]),
    "rram_concat_copy": (I, [P, P, I, I, I, I, I, P]),
    "rram_euclidean_loss_fwd": (I, [P, P, P, P, I64, I, P]),
    "rram_euclidean_loss_bwd": (I, [P, P, I64, F, P]),
    "rram_i32_to_f32": (I, [P, P, I64, P]),
    "rram_dropout_fwd": (I, [P, P, P, I64, F, U64, U32, U64, P]),
    "rram_dropout_bwd": (I, [P, P, P, I64, F, P]),
    "rram_bias_add": (I, [P, P, I, I, I, P]),
    "rram_bias_bwd": (I, [P, P, I, I, I, P]),
    "rram_fill_uniform": (I, [P, I64, F, F, U64, U32, P]),
    "rram_fill_gaussian": (I, [P, I64, F, F, U64, U32, P]),
    "rram_fill_uniform_int": (I, [P, I64, I, F, U64, U32, P]),
}

_lib = None


def load() -> C.CDLL:
    """Load librram_kernels.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not KERNELS_SO.exists():
        raise RramError(f"{KERNELS_SO} not built: run `make -C rram-caffe-simulation_amd` "
                        "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(str(KERNELS_SO), mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc != RRAM_OK:
        msg = load().rram_last_error().decode(errors="replace")
        raise RramError(f"{what or 'rram call'} failed ({rc}): {msg}")


# ---------------------------------------------------------------- thresholds
def prob_threshold(p: float) -> int:
    """32-bit word threshold: r < thr  <=>  u = r / 2^32 < p (exact for dyadic p)."""
    if not (0.0 <= p <= 1.0):
        raise ValueError(f"probability {p} outside [0, 1]")
    return min(TWO32, int(math.ceil(p * TWO32)))


def split_thresholds(neg: int, zero: int, pos: int) -> tuple[int, int]:
    """(thr_neg, thr_zero) for the reference's FailureProbParameter split
    (failure_maker.cpp:10-24): split1 = neg/sum, split2 = (neg+zero)/sum,
    as exact ceilings of split * 2^32."""
    if min(neg, zero, pos) < 0:
        raise ValueError("failure_prob entries must be >= 0 (failure_maker.cpp:11-13)")
    s = neg + zero + pos
    if s <= 0:
        raise ValueError("failure_prob entries sum to 0")
    return (-(-neg * TWO32 // s), -(-(neg + zero) * TWO32 // s))


def gaussian_fault_rate(mean: float, std: float) -> float:
    """P(endurance <= 0) for endurance ~ N(mean, std): the fraction of cells the
    reference's first Fail() pins (failure_maker.cpp:64-66)."""
    if std <= 0:
        return 1.0 if mean <= 0 else 0.0
    return 0.5 * math.erfc(mean / (std * math.sqrt(2.0)))


def mean_for_fault_rate(p: float, std: float) -> float:
    """Inverse of gaussian_fault_rate: mean = -Phi^{-1}(p) * std."""
    from statistics import NormalDist
    return -NormalDist().inv_cdf(p) * std


def make_inject_cfg(p_fault: float, neg: int = 10, zero: int = 20, pos: int = 10, *,
                    stuck_scale: float = 1.0, quant_levels: int = 0, g_max: float = 0.0,
                    var_sigma: float = 0.0, cell_mode: int = RRAM_CELL_SINGLE,
                    p_sa1: float = 0.5) -> InjectCfg:
    tn, tz = split_thresholds(neg, zero, pos)
    return InjectCfg(prob_threshold(p_fault), tn, tz, prob_threshold(p_sa1), stuck_scale, g_max,
                     quant_levels, var_sigma, cell_mode, 0)
