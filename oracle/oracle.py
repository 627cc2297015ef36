"""Python face of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline; the product
(rram-caffe-simulation_amd/) never does.

Two layers:
  * ctypes binding of oracle.c (the fault arithmetic, Philox, GEMM, im2col,
    conv — exact C restatements of the reference, see file header there);
  * numpy restatements of the reference's CPU layer code for the support
    layers and a Caffe-CPU-mode network forward (per-image im2col + sgemm via
    numpy's OpenBLAS) used as the CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import math
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SO = HERE / "_build" / "liboracle.so"

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not SO.exists():
            build()
        L = C.CDLL(str(SO))
        P, I, I64, U32, U64, F = C.c_void_p, C.c_int, C.c_int64, C.c_uint32, C.c_uint64, C.c_float
        L.oracle_philox.argtypes = [P, P, P]
        L.oracle_fault_threshold.argtypes = [P, I64, F, F]
        L.oracle_fault_init.argtypes = [P, P, I64, F, F, U64, U64, U64, U32, U32]
        L.oracle_fail_apply.argtypes = [P, P, P, P, I64, F, F]
        L.oracle_fail_apply.restype = I64
        L.oracle_inject.argtypes = [P, P, I64, P, U64, U32, U32]
        L.oracle_inject.restype = I64
        L.oracle_threshold.argtypes = [P, I64, F]
        L.oracle_threshold.restype = I64
        L.oracle_sgd_update.argtypes = [P, P, I64, F, F]
        L.oracle_fused_update_fail.argtypes = [P, P, P, P, P, I64, F, F, F, I, F, F, F]
        L.oracle_fused_update_fail.restype = I64
        L.oracle_gemm.argtypes = [I, I, I, I, I, F, P, P, F, P]
        L.oracle_im2col.argtypes = [P] + [I] * 11 + [P]
        L.oracle_col2im.argtypes = [P] + [I] * 11 + [P]
        L.oracle_conv.argtypes = [P, I, I, I, I, P, P] + [I] * 10 + [P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


def f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


class InjectCfg(C.Structure):  # == rram_inject_cfg
    _fields_ = [
        ("thr_fault", C.c_uint64), ("thr_neg", C.c_uint64), ("thr_zero", C.c_uint64),
        ("thr_sa1", C.c_uint64), ("stuck_scale", C.c_float), ("g_max", C.c_float),
        ("quant_levels", C.c_int32), ("var_sigma", C.c_float), ("cell_mode", C.c_int32),
        ("reserved", C.c_int32),
    ]


# --------------------------------------------------------------- fault model
def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().oracle_philox(c, k, o)
    return list(o)


def fault_threshold(u, split1, split2):
    v = f32(u).copy()
    lib().oracle_fault_threshold(_ptr(v), v.size, split1, split2)
    return v


def fault_init(n, mean, std, thr_neg, thr_zero, seed, map_id=0, layer_id=0):
    e = np.empty(n, np.float32)
    v = np.empty(n, np.float32)
    lib().oracle_fault_init(_ptr(e), _ptr(v), n, mean, std, thr_neg, thr_zero, seed, map_id,
                            layer_id)
    return e, v


def fail_apply(dw, w, e, v, decrement=100.0, eps=1e-20):
    """Returns (w', e', broken_count); inputs are not modified."""
    dw, v = f32(dw), f32(v)
    w, e = f32(w).copy(), f32(e).copy()
    nb = lib().oracle_fail_apply(_ptr(dw), _ptr(w), _ptr(e), _ptr(v), w.size, decrement, eps)
    return w, e, nb


def inject(src, cfg: InjectCfg, seed, map_id, layer_id):
    src = f32(src)
    dst = np.empty_like(src)
    nb = lib().oracle_inject(_ptr(src), _ptr(dst), src.size, C.byref(cfg), seed, map_id, layer_id)
    return dst, nb


def threshold(dw, thr):
    d = f32(dw).copy()
    n = lib().oracle_threshold(_ptr(d), d.size, thr)
    return d, n


def sgd_update(g, h, momentum, lr):
    g, h = f32(g).copy(), f32(h).copy()
    lib().oracle_sgd_update(_ptr(g), _ptr(h), g.size, momentum, lr)
    return g, h


def fused_update_fail(w, g, h, e, v, decay, mom, lr, apply_thr, thr, dec=100.0, eps=1e-20):
    w, g, h = f32(w).copy(), f32(g).copy(), f32(h).copy()
    if e is not None:
        e, v = f32(e).copy(), f32(v)
        ep, vp = _ptr(e), _ptr(v)
    else:
        ep = vp = None
    nb = lib().oracle_fused_update_fail(_ptr(w), _ptr(g), _ptr(h), ep, vp, w.size, decay, mom, lr,
                                        int(apply_thr), thr, dec, eps)
    return w, g, h, e, nb


# ------------------------------------------------------------------ GEMM/conv
def gemm(ta, tb, M, N, K, alpha, A, B, beta=0.0, Cm=None):
    A, B = f32(A), f32(B)
    out = np.zeros(M * N, np.float32) if Cm is None else f32(Cm).copy().reshape(-1)
    lib().oracle_gemm(int(ta), int(tb), M, N, K, alpha, _ptr(A), _ptr(B), beta, _ptr(out))
    return out.reshape(M, N)


def out_size(h, k, p, s, d=1):
    return (h + 2 * p - (d * (k - 1) + 1)) // s + 1


def im2col(im, kh, kw, ph, pw, sh, sw, dh=1, dw=1):
    im = f32(im)
    Cc, H, W = im.shape
    Ho, Wo = out_size(H, kh, ph, sh, dh), out_size(W, kw, pw, sw, dw)
    col = np.empty((Cc * kh * kw, Ho * Wo), np.float32)
    lib().oracle_im2col(_ptr(im), Cc, H, W, kh, kw, ph, pw, sh, sw, dh, dw, _ptr(col))
    return col


def col2im(col, Cc, H, W, kh, kw, ph, pw, sh, sw, dh=1, dw=1):
    col = f32(col)
    im = np.empty((Cc, H, W), np.float32)
    lib().oracle_col2im(_ptr(col), Cc, H, W, kh, kw, ph, pw, sh, sw, dh, dw, _ptr(im))
    return im


def conv_naive(x, w, b, stride=1, pad=0, dilation=1, group=1):
    """caffe_conv restatement (test_convolution_layer.cpp:21-139)."""
    x, w = f32(x), f32(w)
    N, Cc, H, W = x.shape
    Cout, _, kh, kw = w.shape
    Ho, Wo = out_size(H, kh, pad, stride, dilation), out_size(W, kw, pad, stride, dilation)
    out = np.zeros((N, Cout, Ho, Wo), np.float32)
    bp = _ptr(f32(b)) if b is not None else None
    lib().oracle_conv(_ptr(x), N, Cc, H, W, _ptr(w), bp, Cout, kh, kw, pad, pad, stride, stride,
                      dilation, dilation, group, _ptr(out))
    return out


# ------------------------------------------------- numpy layer restatements
def conv_im2col(x, w, b, stride=1, pad=0, dilation=1, group=1):
    """Caffe CPU-mode convolution: per image im2col_cpu + one sgemm per group
    (base_conv_layer.cpp:256-290, conv_layer.cpp:7-24) on numpy/OpenBLAS."""
    x, w = f32(x), f32(w)
    N, Cc, H, W = x.shape
    Cout, cg, kh, kw = w.shape
    Ho, Wo = out_size(H, kh, pad, stride, dilation), out_size(W, kw, pad, stride, dilation)
    out = np.empty((N, Cout, Ho * Wo), np.float32)
    og = Cout // group
    wm = w.reshape(group, og, cg * kh * kw)
    for n in range(N):
        col = im2col_np(x[n], kh, kw, pad, pad, stride, stride, dilation, dilation)
        col = col.reshape(group, cg * kh * kw, Ho * Wo)
        for g in range(group):
            out[n, g * og:(g + 1) * og] = wm[g] @ col[g]
    if b is not None:
        out += f32(b)[None, :, None]
    return out.reshape(N, Cout, Ho, Wo)


def im2col_np(im, kh, kw, ph, pw, sh, sw, dh=1, dw=1):
    """Vectorised numpy im2col with the same [C*kh*kw][Ho*Wo] layout (im2col.cpp:18-55)."""
    Cc, H, W = im.shape
    Ho, Wo = out_size(H, kh, ph, sh, dh), out_size(W, kw, pw, sw, dw)
    p = np.zeros((Cc, H + 2 * ph, W + 2 * pw), np.float32)
    p[:, ph:ph + H, pw:pw + W] = im
    cols = np.empty((Cc, kh, kw, Ho, Wo), np.float32)
    for a in range(kh):
        for b in range(kw):
            cols[:, a, b] = p[:, a * dh:a * dh + sh * (Ho - 1) + 1:sh,
                              b * dw:b * dw + sw * (Wo - 1) + 1:sw]
    return cols.reshape(Cc * kh * kw, Ho * Wo)


def pool_out(h, k, p, s):
    """pooling_layer.cpp:90-104 (ceil rule + clip when padded)."""
    o = int(math.ceil((h + 2 * p - k) / s)) + 1
    if p and (o - 1) * s >= h + p:
        o -= 1
    return o


def pool(x, k, s, p=0, method="MAX"):
    x = f32(x)
    N, Cc, H, W = x.shape
    PH, PW = pool_out(H, k, p, s), pool_out(W, k, p, s)
    out = np.empty((N, Cc, PH, PW), np.float32)
    for a in range(PH):
        for b in range(PW):
            hs, ws = a * s - p, b * s - p
            if method == "MAX":
                he, we = min(hs + k, H), min(ws + k, W)
                hs, ws = max(hs, 0), max(ws, 0)
                out[:, :, a, b] = x[:, :, hs:he, ws:we].max(axis=(2, 3))
            else:
                he, we = min(hs + k, H + p), min(ws + k, W + p)
                size = (he - hs) * (we - ws)
                hs, ws, he, we = max(hs, 0), max(ws, 0), min(he, H), min(we, W)
                out[:, :, a, b] = x[:, :, hs:he, ws:we].sum(axis=(2, 3)) / size
    return out


def lrn(x, size, alpha, beta, k=1.0):
    """lrn_layer.cpp CrossChannelForward_cpu: scale = k + alpha/size * sum x^2."""
    x = f32(x)
    N, Cc, H, W = x.shape
    pre = (size - 1) // 2
    sq = np.zeros((N, Cc + size - 1, H, W), np.float32)
    sq[:, pre:pre + Cc] = x * x
    scale = np.full(x.shape, k, np.float32)
    for c in range(Cc):
        scale[:, c] += (alpha / size) * sq[:, c:c + size].sum(axis=1)
    return x * np.power(scale, -beta)


def lrn_within(x, size, alpha, beta):
    """lrn_layer.cpp WithinChannelForward (lines 155-163 + the LayerSetUp sub-net
    at 17-62): square -> AVE pool(size, pad (size-1)/2, stride 1) -> power
    (1 + alpha * avg)^-beta -> eltwise product with x."""
    x = f32(x)
    pre = (size - 1) // 2
    avg = pool(x * x, size, 1, pre, "AVE")
    return (x * np.power(np.float32(1.0) + np.float32(alpha) * avg, np.float32(-beta))).astype(np.float32)


def relu(x, slope=0.0):
    x = f32(x)
    return np.where(x > 0, x, x * slope).astype(np.float32)


def softmax(x):
    x = f32(x)
    m = x.max(axis=1, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=1, keepdims=True)


def accuracy(x, label, top_k=1):
    """accuracy_layer.cpp:48-90: (value, index) pairs, descending, top_k."""
    x = f32(x).reshape(len(label), -1)
    correct = 0
    for i, lv in enumerate(np.asarray(label, dtype=np.int64)):
        v = x[i, lv]
        rank = int(np.sum((x[i] > v) | ((x[i] == v) & (np.arange(x.shape[1]) > lv))))
        correct += rank < top_k
    return correct


def softmax_loss(prob, label):
    p = prob[np.arange(len(label)), np.asarray(label, np.int64)]
    return float(-np.log(np.maximum(p, np.finfo(np.float32).tiny)).sum() / len(label))


# ----------------------------------------------------------------------------
# Fault-tolerance strategies (src/caffe/strategy.cpp) — numpy / pure-Python
# restatements for small nets.  The reference sorts with std::sort (unstable);
# callers give inputs whose sort keys are distinct, so argsort is the same order.
# ----------------------------------------------------------------------------
def remap_orders(e_list, v_list):
    """SortFCNeurons (strategy.cpp:48-86): e_list / v_list are the fault states
    of the FC weight blobs (2-D, in fc_params_ids_ order)."""
    flags = [((e < 0) & (v == 0)).astype(np.int64) for e, v in zip(e_list, v_list)]  # GetFailFlagMat :36-45
    orders = []
    for i in range(1, len(flags)):
        zero_nums = flags[i - 1].sum(axis=1) + flags[i].sum(axis=0)   # asum row + strided asum column
        assert len(np.unique(zero_nums)) == len(zero_nums), "oracle needs distinct sort keys"
        orders.append(np.argsort(zero_nums, kind="stable"))
    return orders


def remap_apply(fc_w, fc_wd, fc_b, fc_bd, e_list, v_list, prune_orders, compat=False):
    """RemappingFailureStrategy::Apply (strategy.cpp:88-137) on copies.
    fc_w/fc_wd: FC weight data/diff (2-D), fc_b/fc_bd: their biases."""
    W = [w.copy() for w in fc_w]
    Wd = [w.copy() for w in fc_wd]
    B = [b.copy() for b in fc_b]
    Bd = [b.copy() for b in fc_bd]
    orders = remap_orders(e_list, v_list)
    for i in range(1, len(W)):
        order, prune = orders[i - 1], np.asarray(prune_orders[i - 1])
        rw, rwd, rb, rbd = W[i - 1].copy(), Wd[i - 1].copy(), B[i - 1].copy(), Bd[i - 1].copy()
        for j in range(len(order)):
            W[i - 1][order[j]] = rw[prune[j]]
            Wd[i - 1][order[j]] = rwd[prune[j]]
            if compat:   # strategy.cpp:118-119 reads the weight array (Appendix A Q8)
                B[i - 1][order[j]] = rw.reshape(-1)[prune[j]]
                Bd[i - 1][order[j]] = rwd.reshape(-1)[prune[j]]
            else:
                B[i - 1][order[j]] = rb[prune[j]]
                Bd[i - 1][order[j]] = rbd[prune[j]]
        ow, owd = W[i].copy(), Wd[i].copy()
        for j in range(len(order)):
            W[i][:, order[j]] = ow[:, prune[j]]
            Wd[i][:, order[j]] = owd[:, prune[j]]
    return W, Wd, B, Bd, orders


def genetic_apply(fc_ids, fail_e, prune, weights, rand, switch_time, compat=False):
    """GeneticFailureStrategy::Apply (strategy.cpp:158-288) on copies.
    fail_e / prune / weights: per failure param (flat arrays; weights as
    (data, diff, shape)); fc_ids: indices of the FC weight params; rand: the
    rand() stream.  Returns (weights', prune', dist_before, dist_after, accepted)."""
    eps = np.float32(1e-20)
    P = [p.astype(np.float32).copy() for p in prune]
    Wt = [(d.copy(), g.copy(), s) for d, g, s in weights]

    def overall():
        return sum(int(((p < eps) & (e < 0)).sum()) for p, e in zip(P, fail_e))
    before = overall()
    size = len(fc_ids)
    accepted = 0
    i = 0
    while i < switch_time:
        li = rand() % (size - 1) + 1
        a, b = fc_ids[li - 1], fc_ids[li]
        layer_dim, in_dim = Wt[a][2]
        n1 = rand() % layer_dim
        n2 = rand() % layer_dim
        if n1 == n2:
            continue
        i += 1
        out_dim = Wt[b][2][0]
        fin = fail_e[a].reshape(layer_dim, in_dim)
        fout = fail_e[b].reshape(out_dim, layer_dim)
        pin = P[a].reshape(layer_dim, in_dim)
        pout = P[b].reshape(out_dim, layer_dim)
        db = int(((pin[n1] < eps) & (fin[n1] < 0)).sum() + ((pin[n2] < eps) & (fin[n2] < 0)).sum()
                 + ((pout[:, n1] < eps) & (fout[:, n1] < 0)).sum() + ((pout[:, n2] < eps) & (fout[:, n2] < 0)).sum())
        da = int(((pin[n2] < eps) & (fin[n1] < 0)).sum() + ((pin[n1] < eps) & (fin[n2] < 0)).sum()
                 + ((pout[:, n2] < eps) & (fout[:, n1] < 0)).sum() + ((pout[:, n1] < eps) & (fout[:, n2] < 0)).sum())
        if da < db:
            accepted += 1
            for arr in (Wt[a][0], Wt[a][1]):
                m = arr.reshape(layer_dim, in_dim)
                m[[n1, n2]] = m[[n2, n1]]
            for arr in (Wt[a + 1][0], Wt[a + 1][1]):   # bias (strategy.cpp:250-255)
                arr[[n1, n2]] = arr[[n2, n1]]
            pin[[n1, n2]] = pin[[n2, n1]]
            if compat:                                   # Appendix A Q9 (strategy.cpp:265-267)
                flat = P[a]
                flat[n1], flat[n2] = flat[n2], flat[n1]
            elif a + 1 < len(P) and P[a + 1].size == layer_dim:
                P[a + 1][[n1, n2]] = P[a + 1][[n2, n1]]
            for arr in (Wt[b][0], Wt[b][1]):
                m = arr.reshape(out_dim, layer_dim)
                m[:, [n1, n2]] = m[:, [n2, n1]]
            pout[:, [n1, n2]] = pout[:, [n2, n1]]
    return Wt, P, before, overall(), accepted


# ----------------------------------------------------------------------------
# Caffe CPU mode in C (caffe_cpu.c) — the CPU baseline of bench.py
# ----------------------------------------------------------------------------
def blas_candidates():
    """BLAS libraries on this host the Caffe-CPU restatement can drive:
    numpy's bundled OpenBLAS (ILP64, scipy_ prefix) first, then an LP64
    cblas_sgemm (MKL runtime)."""
    import glob
    import os
    out = []
    for d in {os.path.join(os.path.dirname(np.__file__), os.pardir, "numpy.libs")}:
        out += [(p, 0, "OpenBLAS (numpy bundled, ILP64)") for p in sorted(glob.glob(os.path.join(d, "libscipy_openblas64_*.so")))]
    for p in ("/opt/conda/lib/libmkl_rt.so", "/opt/conda/lib/libmkl_rt.so.1"):
        if os.path.exists(p):
            out.append((p, 1, "MKL runtime (LP64 cblas_sgemm)"))
    return out


_cc_ready = None


def cc_init(threads):
    """Bind caffe_cpu.c to the first loadable BLAS; returns its description."""
    global _cc_ready
    L = lib()
    P, I, I64, F = C.c_void_p, C.c_int, C.c_int64, C.c_float
    L.cc_init.argtypes = [C.c_char_p, I, I]
    L.cc_init.restype = I
    L.cc_gemm.argtypes = [I, I, I, I, I, F, P, P, F, P]
    L.cc_conv_forward.argtypes = [P, I, I, I, I, P, P, I, I, I, I, I, P, P, P]
    L.cc_ip_forward.argtypes = [P, I, I, P, P, I, P, P]
    L.cc_relu.argtypes = [P, I64]
    L.cc_lrn.argtypes = [P, P, I, I, I, I, I, F, F, F, P, P]
    L.cc_maxpool.argtypes = [P, P, P, I, I, I, I, I, I]
    L.cc_softmax.argtypes = [P, P, I, I]
    L.cc_pool.argtypes = [P, P, I, I, I, I, I, I, I, I, I, I]
    for path, mode, desc in blas_candidates():
        if L.cc_init(path.encode(), mode, int(threads)) == 0:
            _cc_ready = desc
            return desc
    raise RuntimeError("no usable BLAS for the Caffe-CPU restatement")


def cc_conv(x, w, b, stride=1, pad=0, group=1):
    x, w = f32(x), f32(w)
    N, Cc, H, W = x.shape
    Cout, cg, k, _ = w.shape
    Ho, Wo = out_size(H, k, pad, stride), out_size(W, k, pad, stride)
    y = np.empty((N, Cout, Ho, Wo), np.float32)
    col = np.empty(Cc * k * k * Ho * Wo, np.float32)
    ones = np.ones(Ho * Wo, np.float32)
    bp = _ptr(f32(b)) if b is not None else None
    lib().cc_conv_forward(_ptr(x), N, Cc, H, W, _ptr(w), bp, Cout, k, pad, stride, group, _ptr(y), _ptr(col),
                          _ptr(ones))
    return y


def cc_ip(x, w, b):
    x, w = f32(x.reshape(len(x), -1)), f32(w)
    M, K = x.shape
    N = w.shape[0]
    y = np.empty((M, N), np.float32)
    ones = np.ones(M, np.float32)
    lib().cc_ip_forward(_ptr(x), M, K, _ptr(w), _ptr(f32(b)) if b is not None else None, N, _ptr(y), _ptr(ones))
    return y


def cc_relu(x):
    x = f32(x)
    lib().cc_relu(_ptr(x), x.size)
    return x


def cc_lrn(x, size, alpha, beta, k=1.0):
    x = f32(x)
    n, c, h, w = x.shape
    y = np.empty_like(x)
    scale = np.empty_like(x)
    padded = np.empty((c + size - 1) * h * w, np.float32)
    lib().cc_lrn(_ptr(x), _ptr(y), n, c, h, w, size, alpha, beta, k, _ptr(scale), _ptr(padded))
    return y


def cc_maxpool(x, k, s):
    x = f32(x)
    n, c, h, w = x.shape
    ph, pw = pool_out(h, k, 0, s), pool_out(w, k, 0, s)
    y = np.empty((n, c, ph, pw), np.float32)
    mask = np.empty((n, c, ph, pw), np.int32)
    lib().cc_maxpool(_ptr(x), _ptr(y), _ptr(mask), n, c, h, w, k, s)
    return y


def cc_pool(x, k, s, p=0, method="MAX"):
    """pooling_layer.cpp Forward_cpu with padding, MAX or AVE (caffe_cpu.c)."""
    x = f32(x)
    n, c, h, w = x.shape
    ph, pw = pool_out(h, k, p, s), pool_out(w, k, p, s)
    y = np.empty((n, c, ph, pw), np.float32)
    lib().cc_pool(_ptr(x), _ptr(y), n, c, h, w, ph, pw, k, s, p, 0 if method == "MAX" else 1)
    return y


def cc_softmax(x):
    x = f32(x.reshape(len(x), -1))
    y = np.empty_like(x)
    lib().cc_softmax(_ptr(x), _ptr(y), x.shape[0], x.shape[1])
    return y


def physical_cores():
    """Physical cores among the CPUs this process may run on: the affinity set
    divided by SMT (one per distinct (package, core) in the sysfs topology)."""
    import os
    cpus = sorted(os.sched_getaffinity(0))
    seen = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology"
        try:
            with open(f"{base}/physical_package_id") as f:
                pkg = f.read().strip()
            with open(f"{base}/core_id") as f:
                core = f.read().strip()
        except OSError:
            return len(cpus)
        seen.add((pkg, core))
    return len(seen) or len(cpus)


def caffe_cpu_alexnet_map(batch=256, p_fault=0.01, seed=1701, threads=None, images=None):
    """One Monte-Carlo fault map of AlexNet b`batch` in Caffe CPU mode
    (SURVEY.md §3.3 / §8d): the GaussianFailureMaker draws for all 58,631,144
    IP cells (mean = -Phi^-1(p)·std so P(endurance <= 0) = p), Fail_cpu at a
    zero update (failure_maker.cpp:55-81: every broken cell takes its stuck
    value), then the TEST forward of `images` (default: all) of the batch in
    the reference's layer order.  Returns (per-layer seconds, metadata)."""
    import os
    import time
    from statistics import NormalDist
    if threads is None:
        threads = physical_cores()
    blas = cc_init(threads)
    rng = np.random.default_rng(seed)
    conv = {"conv1": (96, 3, 11, 4, 0, 1), "conv2": (256, 48, 5, 1, 2, 2), "conv3": (384, 256, 3, 1, 1, 1),
            "conv4": (384, 192, 3, 1, 1, 2), "conv5": (256, 192, 3, 1, 1, 2)}
    w = {k: (rng.standard_normal((co, ci, kk, kk)) * 0.01).astype(np.float32) for k, (co, ci, kk, *_r) in conv.items()}
    b = {k: np.full(conv[k][0], 0.1, np.float32) for k in conv}
    fcs = {"fc6": (4096, 9216, 0.005), "fc7": (4096, 4096, 0.005), "fc8": (1000, 4096, 0.01)}
    fw = {k: (rng.standard_normal(s[:2]) * s[2]).astype(np.float32) for k, s in fcs.items()}
    fb = {k: np.full(s[0], 0.1, np.float32) for k, s in fcs.items()}
    n_img = batch if images is None else images
    x = (rng.integers(0, 256, (n_img, 3, 227, 227)) - 128).astype(np.float32)
    # warm the BLAS thread pool (its first call spawns the threads), untimed
    cc_conv(x[:1], w["conv1"], b["conv1"], 4, 0, 1)
    t = {}
    std = 1e6
    mean = -NormalDist().inv_cdf(p_fault) * std
    neg, zero, tot = 10, 20, 40
    thr_neg = (neg * (1 << 32) + tot - 1) // tot
    thr_zero = ((neg + zero) * (1 << 32) + tot - 1) // tot
    t0 = time.perf_counter()
    broken = 0
    lid = 0
    for k in fcs:
        for arr in (fw, fb):
            a = arr[k].reshape(-1)
            e, v = fault_init(a.size, mean, std, thr_neg, thr_zero, seed, 0, lid)
            dw = np.zeros_like(a)
            nw, _, nb = fail_apply(dw, a, e, v)
            arr[k] = nw.reshape(arr[k].shape)
            broken += nb
            lid += 1
    t["fault map (ctor draws + Fail_cpu)"] = time.perf_counter() - t0

    def tick(name, fn, *a):
        s = time.perf_counter()
        r = fn(*a)
        t[name] = t.get(name, 0.0) + time.perf_counter() - s
        return r

    y = tick("conv1", cc_conv, x, w["conv1"], b["conv1"], 4, 0, 1)
    y = tick("relu1", cc_relu, y)
    y = tick("norm1", cc_lrn, y, 5, 1e-4, 0.75)
    y = tick("pool1", cc_maxpool, y, 3, 2)
    for i, k in enumerate(("conv2", "conv3", "conv4", "conv5"), start=2):
        co, ci, kk, s, p, g = conv[k]
        y = tick(k, cc_conv, y, w[k], b[k], s, p, g)
        y = tick(f"relu{i}", cc_relu, y)
        if k == "conv2":
            y = tick("norm2", cc_lrn, y, 5, 1e-4, 0.75)
            y = tick("pool2", cc_maxpool, y, 3, 2)
    y = tick("pool5", cc_maxpool, y, 3, 2)
    for i, k in enumerate(fcs, start=6):
        y = tick(k, cc_ip, y, fw[k], fb[k])
        if k != "fc8":
            y = tick(f"relu{i}", cc_relu, y)
    prob = tick("prob (softmax)", cc_softmax, y)
    meta = dict(blas=blas, threads=threads, affinity_cpus=len(os.sched_getaffinity(0)),
                physical_cores=physical_cores(), images=n_img,
                broken_cells=broken, finite=bool(np.isfinite(prob).all()))
    return t, meta
