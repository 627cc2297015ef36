"""The bf16x6 engine at the ends of the fp32 range (include/rram_kernels.h,
DESIGN §4.1 "Range").  Every split clamps each term's input to +-BF16_MAX, so
operands above the largest bf16 and +-Inf give the products fp32 gives (+-Inf,
Inf * 0 = NaN; the conv1 kernel's padded K items read zeroed B values, so no
0 * Inf product exists that fp32 does not form); operands down to 2^-110
split exactly (below it the low terms fall under the normal range: the
engine's documented limit, measured by scripts/x6_range_probe.py).  Checked on every
kernel of the engine — the channel-octet convolution, the persistent conv1
kernel, the patch kernel, the GoogLeNet conv1 kernel and the InnerProduct GEMM —
against a CPU float32 evaluation (NaN / +Inf / -Inf positions) and a float64
one (finite outputs within 1e-4 of sum |a*b|)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CONVS = {
    "octet": ((2, 256, 13, 13), 384, 3, 1, 1),
    "conv1": ((2, 3, 227, 227), 96, 11, 4, 0),
    "patch": ((2, 24, 20, 20), 96, 3, 1, 1),
    "conv7s2": ((2, 3, 224, 224), 64, 7, 2, 3),
}


def _cases(xs, ws, seed):
    import torch
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(*xs, generator=g)
    w = torch.randn(*ws, generator=g) * 0.05
    xi = x.clone()
    xi.view(-1)[::997] = float("inf")
    xi.view(-1)[5::1993] = -float("inf")
    wz = w.clone()
    wz.view(-1)[::7] = 0.0
    return {
        "inf_inputs": (xi, w),
        "inf_inputs_zero_weights": (xi, wz),
        "inf_weights": (x, torch.where(torch.arange(w.numel()).reshape(w.shape) % 1009 == 0,
                                       torch.full_like(w, float("inf")), w)),
        "above_bf16_max": (torch.where(x > 2.0, torch.full_like(x, 3.401e38), x), w * 1e-3),
        "large_1e36": (x * 1e36, w),
        "small_2m100": (x * 2.0 ** -100, w),
        "small_2m110_big_w": (x * 2.0 ** -110, w * 2.0 ** 60),
    }


def _compare(got, ref64, mag, r32, what):
    import torch
    got = got.cpu()
    assert torch.equal(torch.isnan(got), torch.isnan(r32)), f"{what}: NaN positions differ"
    assert torch.equal(torch.isposinf(got), torch.isposinf(r32)), f"{what}: +Inf positions differ"
    assert torch.equal(torch.isneginf(got), torch.isneginf(r32)), f"{what}: -Inf positions differ"
    fin = torch.isfinite(r32) & torch.isfinite(ref64) & torch.isfinite(mag)
    err = ((got.double() - ref64).abs() / mag.clamp_min(1e-300))[fin]
    if err.numel():
        assert float(err.max()) <= 1e-4, f"{what}: max err {float(err.max()):.3e} of sum|a*b|"


@pytest.mark.parametrize("kern", list(CONVS))
@pytest.mark.parametrize("case", ["inf_inputs", "inf_inputs_zero_weights", "inf_weights", "above_bf16_max",
                                  "large_1e36", "small_2m100", "small_2m110_big_w"])
def test_conv_range(device, kern, case):
    import torch
    import torch.nn.functional as F
    from rramsim import ops
    xs, co, k, s, p = CONVS[kern]
    x, w = _cases(xs, (co, xs[1], k, k), 3)[case]
    d = ops.conv_desc(xs, co, k, s, p, 1, 1)
    assert ops.f32_engine_for_conv(d) == ops.ENGINE_BF16X6
    y = torch.empty(xs[0], co, d.out_h, d.out_w, device=device)
    ops.conv2d_fwd(d, x.to(device), w.to(device), None, y)
    torch.cuda.synchronize()
    # explicit zero padding: Caffe's im2col multiplies the padded zeros too
    # (0 * Inf = NaN), which a convolution library may skip
    xp = F.pad(x, (p, p, p, p))
    ref = F.conv2d(xp.double(), w.double(), stride=s)
    mag = F.conv2d(xp.double().abs(), w.double().abs(), stride=s)
    r32 = F.conv2d(xp, w, stride=s)
    _compare(y, ref, mag, r32, f"{kern} {case}")


@pytest.mark.parametrize("case", ["inf_inputs", "inf_inputs_zero_weights", "inf_weights", "above_bf16_max",
                                  "large_1e36", "small_2m100", "small_2m110_big_w"])
def test_ip_range(device, case):
    """fc6 shape (256 x 9216 -> 4096) on k_gemm_x6."""
    import torch
    from rramsim import ops
    M, N, K = 256, 4096, 9216
    assert ops.f32_engine_for_ip(M, N, K) == ops.ENGINE_BF16X6
    x, w = _cases((M, K), (N, K), 5)[case]
    y = torch.empty(M, N, device=device)
    ws = torch.empty(256 << 20, dtype=torch.uint8, device=device)
    ops.ip_fwd(x.to(device), w.to(device), None, y, M, N, K, workspace=ws)
    torch.cuda.synchronize()
    _compare(y, x.double() @ w.double().T, x.double().abs() @ w.double().abs().T, x @ w.T, f"ip {case}")
