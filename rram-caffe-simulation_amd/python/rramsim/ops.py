"""Thin torch-tensor wrappers over the C-ABI (device memory via torch, calls
via ctypes).  Every op launches on torch's current HIP stream and raises
RramError on a non-zero status.  No CPU fallback: tensors must live on the GPU.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _kernels as K


def _lib():
    return K.load()


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise K.RramError("rramsim ops take device tensors (no CPU fallback)")
    if t.dtype not in (torch.float32, torch.int32, torch.int64, torch.uint64, torch.uint8):
        raise K.RramError(f"unsupported dtype {t.dtype}")
    return C.c_void_p(t.data_ptr())


def _f32(t, name):
    if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
        raise K.RramError(f"{name} must be a contiguous float32 tensor")


def counters(n: int, device="cuda") -> torch.Tensor:
    return torch.zeros(n, dtype=torch.int64, device=device)


def fault_threshold(values, split1, split2):
    _f32(values, "values")
    K.check(_lib().rram_fault_threshold(_p(values), values.numel(), split1, split2, _stream()),
            "fault_threshold")


def fault_init(endurance, values, mean, std, thr_neg, thr_zero, seed, map_id=0, layer_id=0):
    _f32(endurance, "endurance")
    _f32(values, "values")
    K.check(_lib().rram_fault_init(_p(endurance), _p(values), endurance.numel(), mean, std,
                                   thr_neg, thr_zero, seed, map_id, layer_id, _stream()),
            "fault_init")


def fail_apply(dw, w, endurance, values, decrement=100.0, eps=1e-20, counter=None):
    for t, nm in ((dw, "dw"), (w, "w"), (endurance, "endurance"), (values, "values")):
        _f32(t, nm)
    K.check(_lib().rram_fail_apply(_p(dw), _p(w), _p(endurance), _p(values), w.numel(),
                                   decrement, eps, _p(counter), _stream()), "fail_apply")


def fail_apply_batched(segs, decrement=100.0, eps=1e-20, counters_t=None):
    arr = (K.FailSeg * len(segs))()
    for i, (dw, w, e, v) in enumerate(segs):
        arr[i] = K.FailSeg(dw.data_ptr(), w.data_ptr(), e.data_ptr(), v.data_ptr(), w.numel())
    K.check(_lib().rram_fail_apply_batched(arr, len(segs), decrement, eps, _p(counters_t),
                                           _stream()), "fail_apply_batched")


def inject(w_clean, w_out, cfg, seed, map_id, layer_id, counter=None):
    _f32(w_clean, "w_clean")
    _f32(w_out, "w_out")
    K.check(_lib().rram_inject_rng(_p(w_clean), _p(w_out), w_clean.numel(), C.byref(cfg), seed,
                                   map_id, layer_id, _p(counter), _stream()), "inject_rng")


def inject_batched(segs, seed, map_id, counters_t=None):
    """segs: list of (w_clean, w_out, layer_id, cfg)."""
    arr = (K.InjectSeg * len(segs))()
    for i, (src, dst, lid, cfg) in enumerate(segs):
        arr[i] = K.InjectSeg(src.data_ptr(), dst.data_ptr(), src.numel(), lid, 0, cfg)
    K.check(_lib().rram_inject_rng_batched(arr, len(segs), seed, map_id, _p(counters_t),
                                           _stream()), "inject_rng_batched")


def stuck_zero_counts(e, v, rows, cols, row_counts, col_counts):
    """row_counts[r] = #(e<0 & v==0) in row r; col_counts[c] += same per column (int32 tensors)."""
    _f32(e, "endurance")
    _f32(v, "values")
    K.check(_lib().rram_stuck_zero_counts(_p(e), _p(v), rows, cols, _p(row_counts), _p(col_counts), _stream()),
            "stuck_zero_counts")


def permute_rows(src, dst, row_len, to, frm):
    K.check(_lib().rram_permute_rows(_p(src), _p(dst), row_len, _p(to), _p(frm), to.numel(), _stream()),
            "permute_rows")


def permute_cols(src, dst, rows, cols, to, frm):
    K.check(_lib().rram_permute_cols(_p(src), _p(dst), rows, cols, _p(to), _p(frm), to.numel(), _stream()),
            "permute_cols")


def permute_elems(src, dst, to, frm):
    K.check(_lib().rram_permute_elems(_p(src), _p(dst), _p(to), _p(frm), to.numel(), _stream()), "permute_elems")


def threshold_strategy(dw, thr, counter=None):
    _f32(dw, "dw")
    K.check(_lib().rram_threshold_strategy(_p(dw), dw.numel(), thr, _p(counter), _stream()),
            "threshold_strategy")


def sgd_update(g, h, momentum, local_rate):
    K.check(_lib().rram_sgd_update(_p(g), _p(h), g.numel(), momentum, local_rate, _stream()),
            "sgd_update")


def axpy(alpha, x, y):
    """y = alpha*x + y (caffe_gpu_axpy, math_functions.cu:65-69)."""
    _f32(x, "x")
    _f32(y, "y")
    if x.numel() != y.numel():
        raise K.RramError("axpy: size mismatch")
    K.check(_lib().rram_axpy(x.numel(), alpha, _p(x), _p(y), _stream()), "axpy")


def fused_update_fail(w, g, h, e, v, decay, momentum, lr, apply_thr, thr, decrement=100.0,
                      eps=1e-20, counter=None):
    K.check(_lib().rram_fused_update_fail(_p(w), _p(g), _p(h), _p(e), _p(v), w.numel(), decay,
                                          momentum, lr, int(apply_thr), thr, decrement, eps,
                                          _p(counter), _stream()), "fused_update_fail")


def fused_update_fail_batched(segs, momentum, decrement=100.0, eps=1e-20):
    """segs: list of (w, g, h, e, v, decay, lr, apply_thr, thr, counter); one launch."""
    arr = (K.UpdateSeg * len(segs))()
    for i, (w, g, h, e, v, decay, lr, apply_thr, thr, counter) in enumerate(segs):
        for t, nm in ((w, "w"), (g, "g"), (h, "h"), (e, "endurance"), (v, "values")):
            _f32(t, nm)
        arr[i] = K.UpdateSeg(_p(w), _p(g), _p(h), _p(e), _p(v), w.numel(), decay, lr, thr, int(apply_thr),
                             _p(counter))
    K.check(_lib().rram_fused_update_fail_batched(arr, len(segs), momentum, decrement, eps, _stream()),
            "fused_update_fail_batched")


def gemm(trans_a, trans_b, M, N, K_, alpha, A, B, beta, Cm):
    K.check(_lib().rram_gemm_f32(int(trans_a), int(trans_b), M, N, K_, alpha, _p(A), _p(B), beta,
                                 _p(Cm), _stream()), "gemm")


def gemm_ex(trans_a, trans_b, M, N, K_, alpha, A, lda, B, ldb, beta, Cm, ldc, bias=None,
            bias_mode=0, relu=False, workspace=None):
    ws = _p(workspace)
    wsb = workspace.numel() * workspace.element_size() if workspace is not None else 0
    K.check(_lib().rram_gemm_f32_ex(int(trans_a), int(trans_b), M, N, K_, alpha, _p(A), lda,
                                    _p(B), ldb, beta, _p(Cm), ldc, _p(bias), bias_mode, int(relu),
                                    ws, wsb, _stream()), "gemm_ex")


def gemv(trans_a, M, N, alpha, A, x, beta, y):
    """y = alpha * op(A) x + beta * y, A [M][N] row-major (caffe_gpu_gemv)."""
    K.check(_lib().rram_gemv_f32(int(trans_a), M, N, alpha, _p(A), _p(x), beta, _p(y), _stream()), "gemv")


def conv_desc(x_shape, num_output, kernel, stride=1, pad=0, dilation=1, group=1):
    kh, kw = (kernel, kernel) if isinstance(kernel, int) else kernel
    sh, sw = (stride, stride) if isinstance(stride, int) else stride
    ph, pw = (pad, pad) if isinstance(pad, int) else pad
    dh, dw = (dilation, dilation) if isinstance(dilation, int) else dilation
    n, c, h, w = x_shape
    d = K.ConvDesc(n, c, h, w, num_output, kh, kw, ph, pw, sh, sw, dh, dw, group, 0, 0)
    K.check(_lib().rram_conv_out_shape(C.byref(d)), "conv_out_shape")
    return d


ENGINE_F32, ENGINE_BF16X6 = 0, 1


def set_f32_engine(engine):
    """Matrix-core engine of the stride-1 3x3 / 5x5 convolution forward
    (rram_set_f32_engine); returns the previous one."""
    prev = _lib().rram_set_f32_engine(int(engine))
    if prev < 0:
        K.check(prev, "set_f32_engine")
    return prev


def get_f32_engine():
    return _lib().rram_get_f32_engine()


def f32_engine_for_conv(d):
    """Engine rram_conv2d_fwd would use for this descriptor now."""
    return _lib().rram_f32_engine_for_conv(C.byref(d))


def f32_engine_for_ip(M, N, K, ws_bytes=256 << 20):
    """Engine rram_ip_fwd (W [N][K], aligned operands) would use now."""
    return _lib().rram_f32_engine_for_ip(int(M), int(N), int(K), int(ws_bytes))


def conv2d_fwd(d, x, w, bias, y, relu=False):
    K.check(_lib().rram_conv2d_fwd(C.byref(d), _p(x), _p(w), _p(bias), _p(y), int(relu),
                                   _stream()), "conv2d_fwd")


def conv2d_fwd_octets(d, x, x_oct, w, bias, y, y_oct, relu=False):
    """rram_conv2d_fwd with channel-octet companions (x_oct / y_oct: uint8
    tensors of 6 bytes per element, or None)."""
    K.check(_lib().rram_conv2d_fwd_octets(C.byref(d), _p(x), _p(x_oct), _p(w), _p(bias), _p(y), _p(y_oct),
                                          int(relu), _stream()), "conv2d_fwd_octets")


def conv_weight_pack_bytes(d):
    """Bytes of the bf16x6 engine's packed-weight companion for d (0: no pack)."""
    return int(_lib().rram_conv_weight_pack_bytes(C.byref(d)))


def conv2d_fwd_cached(d, x, x_oct, w, w_pack, w_pack_valid, bias, y, y_oct=None, relu=False):
    """rram_conv2d_fwd_octets with a packed-weight companion w_pack (uint8
    tensor of conv_weight_pack_bytes(d) bytes): w_pack_valid False packs w
    into it first, True uses it as is."""
    K.check(_lib().rram_conv2d_fwd_cached(C.byref(d), _p(x), _p(x_oct), _p(w), _p(w_pack), int(bool(w_pack_valid)),
                                          _p(bias), _p(y), _p(y_oct), int(relu), _stream()), "conv2d_fwd_cached")


def conv2d_fwd_strided(d, x, w, bias, y, y_image_stride, relu=False, x_oct=None, w_pack=None, w_pack_valid=False):
    """rram_conv2d_fwd_strided: image n's output at y + n * y_image_stride
    floats (y may be a channel-offset view into a larger NCHW tensor)."""
    K.check(_lib().rram_conv2d_fwd_strided(C.byref(d), _p(x), _p(x_oct), _p(w), _p(w_pack), int(bool(w_pack_valid)),
                                           _p(bias), C.c_void_p(y.data_ptr()), int(y_image_stride), int(relu),
                                           _stream()), "conv2d_fwd_strided")


def conv_output_octets_only(d):
    """1 when rram_conv2d_fwd_octets accepts y = None with y_oct for d now
    (the channel-octet epilogue writes only the companion)."""
    return _lib().rram_conv_output_octets_only(C.byref(d))


def conv_input_octets(d):
    """1 when rram_conv2d_fwd_octets would read an input companion for d now."""
    return _lib().rram_conv_input_octets(C.byref(d))


def conv_octet_plan(d):
    """The channel-octet kernel's host plan for d: dict(rows, cols, per_cu,
    tiles_per_image, pieces), or None when that kernel does not take d."""
    plan = (C.c_int * 5)()
    if not _lib().rram_conv_octet_plan(C.byref(d), plan):
        return None
    return dict(rows=plan[0], cols=plan[1], per_cu=plan[2], tiles_per_image=plan[3], pieces=plan[4])


def pack_octets(x, oct_, n, c, h, w):
    K.check(_lib().rram_pack_octets(_p(x), _p(oct_), n, c, h, w, _stream()), "pack_octets")


def conv2d_bwd(d, x, w, dy, dw=None, db=None, dx=None, workspace=None):
    wsb = workspace.numel() * workspace.element_size() if workspace is not None else 0
    K.check(_lib().rram_conv2d_bwd(C.byref(d), _p(x), _p(w), _p(dy), _p(dw), _p(db), _p(dx),
                                   _p(workspace), wsb, _stream()), "conv2d_bwd")


def conv2d_bwd_workspace(d, images):
    return _lib().rram_conv2d_bwd_workspace(C.byref(d), images)


def im2col(im, C_, H, W, kh, kw, ph, pw, sh, sw, dh, dw, col):
    K.check(_lib().rram_im2col(_p(im), C_, H, W, kh, kw, ph, pw, sh, sw, dh, dw, _p(col),
                               _stream()), "im2col")


def col2im(col, C_, H, W, kh, kw, ph, pw, sh, sw, dh, dw, im):
    K.check(_lib().rram_col2im(_p(col), C_, H, W, kh, kw, ph, pw, sh, sw, dh, dw, _p(im),
                               _stream()), "col2im")


def ip_fwd(x, w, bias, y, M, N, K_, transpose=False, relu=False, workspace=None):
    wsb = workspace.numel() * workspace.element_size() if workspace is not None else 0
    K.check(_lib().rram_ip_fwd(_p(x), _p(w), _p(bias), _p(y), M, N, K_, int(transpose), int(relu),
                               _p(workspace), wsb, _stream()), "ip_fwd")


def ip_rows_pack_bytes(M, N, K_, ws_bytes):
    """(bytes, rows per tile) of the bf16x6 engine's packed-row input form (0, 0: not served)."""
    bmc = C.c_int(0)
    b = _lib().rram_ip_rows_pack_bytes(M, N, K_, ws_bytes, C.byref(bmc))
    return b, bmc.value


def ip_fwd_rows(x, x_rows, w, bias, y, y_rows, y_rows_per_tile, M, N, K_, relu=False, workspace=None):
    """rram_ip_fwd_rows: returns whether y_rows was written."""
    wsb = workspace.numel() * workspace.element_size() if workspace is not None else 0
    written = C.c_int(0)
    K.check(_lib().rram_ip_fwd_rows(_p(x), _p(x_rows), _p(w), _p(bias), _p(y), _p(y_rows), y_rows_per_tile, M, N,
                                    K_, int(relu), _p(workspace), wsb, C.byref(written), _stream()), "ip_fwd_rows")
    return bool(written.value)


def ip_bwd(x, w, dy, dw, db, dx, M, N, K_, transpose=False):
    K.check(_lib().rram_ip_bwd(_p(x), _p(w), _p(dy), _p(dw), _p(db), _p(dx), M, N, K_,
                               int(transpose), _stream()), "ip_bwd")


def pool_fwd(x, y, mask, geom, method):
    K.check(_lib().rram_pool_fwd(_p(x), _p(y), _p(mask), *geom, method, _stream()), "pool_fwd")


def pool_relu_bwd(dy, mask, dx, geom, method, relu_y, slope):
    """pool_bwd then the in-place ReLU's backward on dx (factor from relu_y), one launch."""
    K.check(_lib().rram_pool_relu_bwd(_p(dy), _p(mask), _p(dx), *geom, method, _p(relu_y), slope, _stream()),
            "pool_relu_bwd")


def pool_relu_fwd(x, y, mask, geom, method, slope):
    """pool_fwd then an in-place ReLU of y, one launch (rram_pool_relu_fwd)."""
    K.check(_lib().rram_pool_relu_fwd(_p(x), _p(y), _p(mask), *geom, method, slope, _stream()), "pool_relu_fwd")


def pool_bwd(dy, mask, dx, geom, method):
    K.check(_lib().rram_pool_bwd(_p(dy), _p(mask), _p(dx), *geom, method, _stream()), "pool_bwd")


def lrn_fwd(x, y, scale, n, c, h, w, size, alpha, beta, k):
    K.check(_lib().rram_lrn_fwd(_p(x), _p(y), _p(scale), n, c, h, w, size, alpha, beta, k,
                                _stream()), "lrn_fwd")


def lrn_bwd(x, y, scale, dy, dx, n, c, h, w, size, alpha, beta):
    K.check(_lib().rram_lrn_bwd(_p(x), _p(y), _p(scale), _p(dy), _p(dx), n, c, h, w, size, alpha,
                                beta, _stream()), "lrn_bwd")


def lrn_maxpool_fwd(x, y, n, c, h, w, ph, pw, kernel, stride, pad, size, alpha, beta, k=1.0):
    K.check(_lib().rram_lrn_maxpool_fwd(_p(x), _p(y), n, c, h, w, ph, pw, kernel, stride, stride, pad, pad,
                                        size, alpha, beta, k, _stream()), "lrn_maxpool_fwd")


def lrn_maxpool_fwd_octets(x, y, y_oct, n, c, h, w, ph, pw, kernel, stride, pad, size, alpha, beta, k=1.0):
    K.check(_lib().rram_lrn_maxpool_fwd_octets(_p(x), _p(y), _p(y_oct), n, c, h, w, ph, pw, kernel, stride, stride,
                                               pad, pad, size, alpha, beta, k, _stream()), "lrn_maxpool_fwd_octets")


def lrn_within_fwd(x, y, scale, n, c, h, w, size, alpha, beta):
    K.check(_lib().rram_lrn_within_fwd(_p(x), _p(y), _p(scale), n, c, h, w, size, alpha, beta,
                                       _stream()), "lrn_within_fwd")


def lrn_within_bwd(x, scale, dy, dx, n, c, h, w, size, alpha, beta):
    K.check(_lib().rram_lrn_within_bwd(_p(x), _p(scale), _p(dy), _p(dx), n, c, h, w, size, alpha,
                                       beta, _stream()), "lrn_within_bwd")


def lrn_within_relu_bwd(x, scale, dy, dx, n, c, h, w, size, alpha, beta, slope):
    """lrn_within_bwd then the in-place ReLU's backward on dx (factor from x), one launch."""
    K.check(_lib().rram_lrn_within_relu_bwd(_p(x), _p(scale), _p(dy), _p(dx), n, c, h, w, size, alpha, beta,
                                            slope, _stream()), "lrn_within_relu_bwd")


def relu_fwd(x, y, slope=0.0):
    K.check(_lib().rram_relu_fwd(_p(x), _p(y), x.numel(), slope, _stream()), "relu_fwd")


def relu_bwd(x, dy, dx, slope=0.0):
    K.check(_lib().rram_relu_bwd(_p(x), _p(dy), _p(dx), x.numel(), slope, _stream()), "relu_bwd")


def softmax_loss_fwd(prob, label, loss, outer, channels, inner, ignore=-1):
    K.check(_lib().rram_softmax_loss_fwd(_p(prob), _p(label), _p(loss), outer, channels, inner, ignore,
                                         _stream()), "softmax_loss_fwd")


def softmax_loss_bwd(prob, label, dx, outer, channels, inner, ignore=-1, loss_weight=1.0):
    K.check(_lib().rram_softmax_loss_bwd(_p(prob), _p(label), _p(dx), outer, channels, inner, ignore,
                                         loss_weight, _stream()), "softmax_loss_bwd")


def softmax_loss_fwd_bwd(prob, label, loss, dx, outer, channels, inner, ignore=-1, loss_weight=1.0):
    """softmax_loss_fwd + softmax_loss_bwd in one launch (<= 65536 elements)."""
    K.check(_lib().rram_softmax_loss_fwd_bwd(_p(prob), _p(label), _p(loss), _p(dx), outer, channels, inner, ignore,
                                             loss_weight, _stream()), "softmax_loss_fwd_bwd")


def concat_copy(src, dst, num, src_cxi, dst_cxi, off_xi, backward=False):
    K.check(_lib().rram_concat_copy(_p(src), _p(dst), num, src_cxi, dst_cxi, off_xi, int(backward),
                                    _stream()), "concat")


def dropout_fwd(x, y, mask, ratio, seed, layer_id=0, it=0):
    K.check(_lib().rram_dropout_fwd(_p(x), _p(y), _p(mask), x.numel(), ratio, seed, layer_id, it,
                                    _stream()), "dropout_fwd")


def dropout_bwd(dy, mask, dx, ratio):
    K.check(_lib().rram_dropout_bwd(_p(dy), _p(mask), _p(dx), dy.numel(), ratio, _stream()), "dropout_bwd")


def softmax_fwd(x, y, outer, channels, inner):
    K.check(_lib().rram_softmax_fwd(_p(x), _p(y), outer, channels, inner, _stream()), "softmax")


def accuracy(x, label, correct, count, outer, channels, inner, top_k=1, ignore=-1, ratio=None):
    K.check(_lib().rram_accuracy(_p(x), _p(label), _p(correct), _p(count), _p(ratio), outer,
                                 channels, inner, top_k, ignore, _stream()), "accuracy")


def fill_uniform(x, lo, hi, seed, sid=0):
    K.check(_lib().rram_fill_uniform(_p(x), x.numel(), lo, hi, seed, sid, _stream()), "fill")


def fill_gaussian(x, mean, std, seed, sid=0):
    K.check(_lib().rram_fill_gaussian(_p(x), x.numel(), mean, std, seed, sid, _stream()), "fill")
