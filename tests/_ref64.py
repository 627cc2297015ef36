"""fp64 layer references with an error scale, for the per-layer parity checks.

Each helper evaluates one Convolution / InnerProduct layer of the reference's
definition (caffe_conv, test_convolution_layer.cpp:21-139; InnerProduct
top = X·Wᵀ + b, inner_product_layer.cpp:83-96) in float64 on the CPU, and
returns it with the layer's error scale Σ|a·b| + |bias| (the same expression
evaluated on absolute values).  A fp32 GEMM of any summation order differs from
the exact value by at most ~K·2^-24 of that scale, so the bound

    |got - ref| <= 1e-4 · scale          (north_star: 1e-4 relative, fp32)

is the scale-aware form of "within 1e-4 relative" that holds for every output
element, including the ones where cancellation makes the plain relative error
meaningless.  Inputs are the GPU's own bottom blobs, so each layer is checked
on its own (no error propagation between layers).
"""
from __future__ import annotations

import numpy as np

TOL = 1e-4


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))


def conv64(x, w, b, stride=1, pad=0, group=1, dilation=1):
    import torch
    F = torch.nn.functional
    x64, w64 = _t(x), _t(w)
    b64 = _t(b) if b is not None else None
    ref = F.conv2d(x64, w64, b64, stride, pad, dilation, group)
    scale = F.conv2d(x64.abs(), w64.abs(), b64.abs() if b is not None else None, stride, pad, dilation, group)
    return ref.numpy(), scale.numpy()


def ip64(x, w, b):
    x64 = np.asarray(x, np.float64).reshape(len(x), -1)
    w64 = np.asarray(w, np.float64).reshape(-1, x64.shape[1])
    ref = x64 @ w64.T
    scale = np.abs(x64) @ np.abs(w64).T
    if b is not None:
        ref = ref + np.asarray(b, np.float64)
        scale = scale + np.abs(np.asarray(b, np.float64))
    return ref, scale


def assert_scaled(got, ref, scale, what, tol=TOL, relu=False):
    got = np.asarray(got, np.float64).reshape(ref.shape)
    if relu:
        ref = np.maximum(ref, 0.0)
    err = np.abs(got - ref)
    bound = tol * scale
    bad = err > bound
    if bad.any():
        r = err / np.maximum(scale, 1e-300)
        i = int(np.argmax(r))
        raise AssertionError(f"{what}: {int(bad.sum())} of {bad.size} elements exceed {tol}·Σ|a·b| "
                             f"(worst err/scale {r.flat[i]:.3e}: got {got.flat[i]!r}, ref {ref.flat[i]!r})")
    return float((err / np.maximum(scale, 1e-300)).max())


def check_conv(got, x, w, b, stride=1, pad=0, group=1, relu=False, what="conv"):
    ref, scale = conv64(x, w, b, stride, pad, group)
    return assert_scaled(got, ref, scale, what, relu=relu)


def check_ip(got, x, w, b, relu=False, what="ip"):
    ref, scale = ip64(x, w, b)
    return assert_scaled(got, ref, scale, what, relu=relu)


def lrn64(x, size, alpha, beta, k=1.0):
    """lrn_layer.cpp CrossChannelForward: x · (k + alpha/size · Σ x²)^-beta, fp64."""
    x = np.asarray(x, np.float64)
    n, c = x.shape[:2]
    pre = (size - 1) // 2
    sq = np.zeros((n, c + size - 1) + x.shape[2:])
    sq[:, pre:pre + c] = x * x
    s = np.full(x.shape, k)
    for ch in range(c):
        s[:, ch] += (alpha / size) * sq[:, ch:ch + size].sum(axis=1)
    return x * np.power(s, -beta)


def maxpool64(x, k, s):
    import math
    x = np.asarray(x, np.float64)
    H, W = x.shape[2:]
    PH = int(math.ceil((H - k) / s)) + 1
    PW = int(math.ceil((W - k) / s)) + 1
    out = np.empty(x.shape[:2] + (PH, PW))
    for a in range(PH):
        for b_ in range(PW):
            out[:, :, a, b_] = x[:, :, a * s:min(a * s + k, H), b_ * s:min(b_ * s + k, W)].max(axis=(2, 3))
    return out


# fp32-level guard of the bf16x6 engine (tests/test_gpu_fp32_guard.py): per
# layer, errors in units of Σ|a·b| (max, mean) of the bf16x6 kernel and of the
# fp32-MFMA kernel on the same data.  The 1e-4 gate above would pass a kernel
# that had lost fp32 accuracy; these bounds do not (tests/test_x6_guard_emulation.py).
X6_GUARD_MAX = 1e-6
X6_GUARD_RATIO = 2.0


def x6_guard_failures(x6, f32):
    """x6, f32 = (max, mean) error / Σ|a·b|; the list of violated bounds."""
    bad = []
    if not x6[0] <= X6_GUARD_MAX:
        bad.append(f"max {x6[0]:.3e} > {X6_GUARD_MAX}")
    if not x6[0] <= X6_GUARD_RATIO * f32[0]:
        bad.append(f"max {x6[0]:.3e} > {X6_GUARD_RATIO} x fp32 MFMA max {f32[0]:.3e}")
    if not x6[1] <= X6_GUARD_RATIO * f32[1]:
        bad.append(f"mean {x6[1]:.3e} > {X6_GUARD_RATIO} x fp32 MFMA mean {f32[1]:.3e}")
    return bad
