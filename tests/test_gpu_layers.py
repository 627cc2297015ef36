"""Support-layer forward/backward kernels against plain PyTorch fp32 references
(autograd for the backward passes).  These are the layers the config nets run
around the conv/IP GEMMs: ReLU, pooling, LRN (both regions), softmax loss,
dropout, concat.  Caffe-specific rules (ceil pooling output, AVE-pool divisor
over the padded window, max-pool first-argmax) are in the references below."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _t(a, device):
    import torch
    return torch.as_tensor(np.ascontiguousarray(a, np.float32)).to(device)


def test_relu_fwd_bwd(device):
    import torch
    from rramsim import ops
    x = torch.randn(4097, device=device)
    dy = torch.randn_like(x)
    for slope in (0.0, 0.1):
        y, dx = torch.empty_like(x), torch.empty_like(x)
        ops.relu_fwd(x, y, slope)
        ops.relu_bwd(x, dy, dx, slope)
        assert torch.equal(y, torch.where(x > 0, x, x * slope))
        assert torch.equal(dx, torch.where(x > 0, dy, dy * slope))


def _caffe_pool_ref(x, k, s, p, method):
    """pooling_layer.cpp:90-104 ceil rule; AVE divides by the window clipped to
    [-pad, H+pad) (pooling_layer.cpp:196-222), MAX ignores the padding."""
    import torch
    import torch.nn.functional as F
    N, C, H, W = x.shape
    PH = -(-(H + 2 * p - k) // s) + 1
    PW = -(-(W + 2 * p - k) // s) + 1
    if p and (PH - 1) * s >= H + p:
        PH -= 1
    if p and (PW - 1) * s >= W + p:
        PW -= 1
    if method == "MAX":
        xp = F.pad(x, (p, p + k, p, p + k), value=-float("inf"))
    else:
        xp = F.pad(x, (p, p + k, p, p + k), value=0.0)
    rows = []
    for a in range(PH):
        cols = []
        for b in range(PW):
            win = xp[:, :, a * s:a * s + k, b * s:b * s + k]
            if method == "MAX":
                cols.append(win.amax(dim=(2, 3)))
            else:
                he, we = min(a * s - p + k, H + p), min(b * s - p + k, W + p)
                size = (he - (a * s - p)) * (we - (b * s - p))
                cols.append(win.sum(dim=(2, 3)) / size)
        rows.append(torch.stack(cols, -1))
    return torch.stack(rows, -2)


@pytest.mark.parametrize("method,k,s,p", [("MAX", 3, 2, 0), ("MAX", 2, 2, 0), ("MAX", 3, 2, 1), ("MAX", 3, 1, 1),
                                          ("AVE", 3, 2, 1), ("AVE", 5, 3, 0), ("AVE", 3, 1, 1)])
def test_pool_fwd_bwd_vs_autograd(device, method, k, s, p):
    import torch
    from rramsim import ops
    torch.manual_seed(3)
    x = torch.randn(2, 5, 13, 11, device=device).requires_grad_(True)
    ref = _caffe_pool_ref(x, k, s, p, method)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    N, C, H, W = x.shape
    geom = (N, C, H, W, ref.shape[2], ref.shape[3], k, k, s, s, p, p)
    y = torch.empty_like(ref)
    mask = torch.empty(ref.shape, dtype=torch.int32, device=device)
    dx = torch.empty_like(x)
    m = 0 if method == "MAX" else 1
    ops.pool_fwd(x.detach(), y, mask, geom, m)
    ops.pool_bwd(dy, mask, dx, geom, m)
    torch.testing.assert_close(y, ref.detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(dx, x.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("shape,k,s,p", [((8, 64, 28, 28), 3, 1, 1), ((4, 48, 27, 27), 3, 2, 0),
                                         ((3, 7, 64, 64), 2, 2, 0), ((2, 9, 7, 7), 3, 2, 1)])
def test_max_pool_plane_kernel_equals_direct(device, shape, k, s, p):
    """The LDS-plane max pool (several planes per block; 64 x 64 planes take
    the direct kernel) against MaxPoolForward restated (pooling_layer.cu:11-47:
    window clipped to the image, -FLT_MAX start, strict ">" in row-major
    order): values and argmax mask, bit for bit."""
    import torch
    from rramsim import ops
    torch.manual_seed(4)
    x = torch.randn(*shape, device=device)
    x[0, 0, :3, :3] = 1.0                            # ties: the first index wins
    N, C, H, W = shape
    PH = -(-(H + 2 * p - k) // s) + 1
    PW = -(-(W + 2 * p - k) // s) + 1
    if (PH - 1) * s >= H + p:
        PH -= 1
    if (PW - 1) * s >= W + p:
        PW -= 1
    geom = (N, C, H, W, PH, PW, k, k, s, s, p, p)
    y = torch.full((N, C, PH, PW), float("nan"), device=device)
    m = torch.full((N, C, PH, PW), -7, dtype=torch.int32, device=device)
    ops.pool_fwd(x, y, m, geom, 0)
    torch.cuda.synchronize()
    xs = x.cpu().numpy()
    ry = np.empty((N, C, PH, PW), np.float32)
    rm = np.empty((N, C, PH, PW), np.int32)
    for a in range(PH):
        for b in range(PW):
            hs, ws = a * s - p, b * s - p
            he, we = min(hs + k, H), min(ws + k, W)
            hs, ws = max(hs, 0), max(ws, 0)
            win = xs[:, :, hs:he, ws:we].reshape(N, C, -1)
            i = win.argmax(axis=2)                    # first maximum in row-major order
            ry[:, :, a, b] = np.take_along_axis(win, i[..., None], 2)[..., 0]
            rm[:, :, a, b] = (hs + i // (we - ws)) * W + ws + i % (we - ws)
    np.testing.assert_array_equal(y.cpu().numpy(), ry)
    np.testing.assert_array_equal(m.cpu().numpy(), rm)


def _max_pool_scan(xs, k, s, p, PH, PW):
    """MaxPoolForward's value (pooling_layer.cu:11-47) restated as a scan:
    window clipped to the image, -FLT_MAX start, strict ">" in row-major order
    (a NaN never wins, the first of equal values (+0 / -0) stays)."""
    N, C, H, W = xs.shape
    out = np.empty((N, C, PH, PW), np.float32)
    for a in range(PH):
        for b in range(PW):
            hs, ws = a * s - p, b * s - p
            he, we = min(hs + k, H), min(ws + k, W)
            hs, ws = max(hs, 0), max(ws, 0)
            m = np.full((N, C), np.finfo(np.float32).min, np.float32)
            for h in range(hs, he):
                for w in range(ws, we):
                    v = xs[:, :, h, w]
                    m = np.where(v > m, v, m)
            out[:, :, a, b] = m
    return out


@pytest.mark.parametrize("shape,s,p", [((3, 64, 28, 28), 1, 1), ((2, 20, 14, 14), 1, 1), ((2, 100, 7, 7), 1, 1),
                                       ((2, 5, 56, 56), 2, 0), ((2, 7, 28, 28), 2, 0), ((3, 6, 13, 11), 2, 1),
                                       ((2, 9, 9, 10), 1, 0), ((1, 3, 129, 127), 2, 1)])
def test_max_pool_sep3_equals_scan(device, shape, s, p):
    """The TEST-phase 3 x 3 max pool without argmax (k_pool_planes_sep3: the
    separable window, several planes per block) against
    MaxPoolForward's scan, bit for bit, with ties of +0 / -0, NaN, +-Inf and
    -FLT_MAX in the input; and the fused-ReLU form against relu() of it."""
    import torch
    from rramsim import ops
    g = torch.Generator().manual_seed(11)
    x = torch.randn(*shape, generator=g)
    flat = x.view(-1)
    n = flat.numel()
    flat[torch.randint(0, n, (n // 50,), generator=g)] = 0.0
    flat[torch.randint(0, n, (n // 50,), generator=g)] = -0.0
    flat[torch.randint(0, n, (n // 200,), generator=g)] = float("nan")
    flat[torch.randint(0, n, (n // 300,), generator=g)] = float("inf")
    flat[torch.randint(0, n, (n // 300,), generator=g)] = -float("inf")
    flat[torch.randint(0, n, (n // 300,), generator=g)] = float(np.finfo(np.float32).min)
    x[0, 0] = -0.0                                   # a plane of signed zeros only
    x[0, 0, 1::3, ::2] = 0.0
    x[-1, -1] = float("nan")                         # all NaN: -FLT_MAX out
    N, C, H, W = shape
    k = 3
    PH = -(-(H + 2 * p - k) // s) + 1
    PW = -(-(W + 2 * p - k) // s) + 1
    if (PH - 1) * s >= H + p:
        PH -= 1
    if (PW - 1) * s >= W + p:
        PW -= 1
    geom = (N, C, H, W, PH, PW, k, k, s, s, p, p)
    ref = _max_pool_scan(x.numpy(), k, s, p, PH, PW)
    xd = x.to(device)
    y = torch.full((N, C, PH, PW), 7.0, device=device)
    ops.pool_fwd(xd, y, None, geom, 0)
    torch.cuda.synchronize()
    assert y.cpu().numpy().tobytes() == ref.tobytes()
    ops.pool_relu_fwd(xd, y, None, geom, 0, 0.0)
    torch.cuda.synchronize()
    torch.testing.assert_close(y.cpu(), torch.relu(torch.from_numpy(ref)), rtol=0, atol=0)


def _lrn_across_ref(x, size, alpha, beta, k):
    import torch.nn.functional as F
    pre = (size - 1) // 2
    sq = F.pad((x * x).unsqueeze(1), (0, 0, 0, 0, pre, size - 1 - pre)).squeeze(1)
    s = sum(sq[:, i:i + x.shape[1]] for i in range(size))
    return x * (k + alpha / size * s) ** (-beta)


def _lrn_within_ref(x, size, alpha, beta):
    import torch.nn.functional as F
    pre = (size - 1) // 2
    avg = F.avg_pool2d(x * x, size, 1, pre, count_include_pad=True)
    return x * (1.0 + alpha * avg) ** (-beta)


@pytest.mark.parametrize("size", [3, 5])
def test_lrn_across_fwd_bwd_vs_autograd(device, size):
    import torch
    from rramsim import ops
    torch.manual_seed(4)
    x = (3 * torch.randn(3, 11, 7, 9, device=device)).requires_grad_(True)
    alpha, beta, k = 1e-2, 0.75, 2.0
    ref = _lrn_across_ref(x, size, alpha, beta, k)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    N, C, H, W = x.shape
    y, sc, dx = torch.empty_like(ref), torch.empty_like(ref), torch.empty_like(ref)
    ops.lrn_fwd(x.detach(), y, sc, N, C, H, W, size, alpha, beta, k)
    ops.lrn_bwd(x.detach(), y, sc, dy, dx, N, C, H, W, size, alpha, beta)
    torch.testing.assert_close(y, ref.detach(), rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(dx, x.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("size,k,s,p,C,H", [(5, 3, 2, 0, 13, 15), (5, 3, 2, 0, 96, 55), (3, 3, 2, 1, 7, 12),
                                             (5, 2, 2, 0, 9, 10), (3, 3, 1, 0, 6, 8), (5, 3, 2, 0, 256, 27),
                                             (5, 2, 1, 1, 5, 21), (3, 3, 3, 2, 4, 30), (5, 3, 2, 1, 6, 33),
                                             (3, 3, 2, 0, 10, 64), (5, 3, 2, 0, 8, 70)])
def test_lrn_maxpool_fused_equals_unfused(device, size, k, s, p, C, H):
    """rram_lrn_maxpool_fwd == rram_lrn_fwd then rram_pool_fwd, bit for bit
    (same LRN arithmetic; window edges of the ceil rule), and the torch fp32
    reference within the LRN tolerance."""
    import torch
    from rramsim import ops
    torch.manual_seed(9)
    N, W = 3, H - 1
    x = 4 * torch.randn(N, C, H, W, device=device)
    alpha, beta, kk = 1e-2, 0.75, 1.5
    lrn = torch.empty_like(x)
    ops.lrn_fwd(x, lrn, None, N, C, H, W, size, alpha, beta, kk)
    ref = _caffe_pool_ref(lrn, k, s, p, "MAX")
    PH, PW = ref.shape[2], ref.shape[3]
    unfused = torch.empty_like(ref)
    ops.pool_fwd(lrn, unfused, None, (N, C, H, W, PH, PW, k, k, s, s, p, p), 0)
    fused = torch.full_like(ref, float("nan"))
    ops.lrn_maxpool_fwd(x, fused, N, C, H, W, PH, PW, k, s, p, size, alpha, beta, kk)
    torch.cuda.synchronize()
    assert torch.equal(fused, unfused)
    torch.testing.assert_close(fused, _caffe_pool_ref(_lrn_across_ref(x, size, alpha, beta, kk), k, s, p, "MAX"),
                               rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize("C,H,N", [(96, 55, 3), (256, 27, 3), (96, 55, 256), (256, 27, 256)])
def test_lrn_maxpool_fused_equals_unfused_alexnet_planes(device, C, H, N):
    """AlexNet's square 55 x 55 / 27 x 27 planes take the band kernel's
    compile-time-width path (immediate-offset pooling taps): bit for bit the
    unfused LRN + max pool, with and without the octet companion.  At b256
    the host cuts both planes' channels into 32-channel chunks, which take the
    straight-line channel walk (N = 3: 8-channel chunks, the loop walk)."""
    import torch
    from rramsim import ops
    torch.manual_seed(11)
    W = H
    x = 4 * torch.randn(N, C, H, W, device=device)
    alpha, beta, kk = 1e-2, 0.75, 1.5
    lrn = torch.empty_like(x)
    ops.lrn_fwd(x, lrn, None, N, C, H, W, 5, alpha, beta, kk)
    PH = PW = (H - 3 + 1) // 2 + 1
    geom = (N, C, H, W, PH, PW, 3, 3, 2, 2, 0, 0)
    unfused = torch.empty((N, C, PH, PW), device=device)
    ops.pool_fwd(lrn, unfused, None, geom, 0)
    fused = torch.full_like(unfused, float("nan"))
    ops.lrn_maxpool_fwd(x, fused, N, C, H, W, PH, PW, 3, 2, 0, 5, alpha, beta, kk)
    fo = torch.full_like(unfused, float("nan"))
    yo = torch.zeros(unfused.numel() * 6, dtype=torch.uint8, device=device)
    ops.lrn_maxpool_fwd_octets(x, fo, yo, N, C, H, W, PH, PW, 3, 2, 0, 5, alpha, beta, kk)
    torch.cuda.synchronize()
    assert torch.equal(fused, unfused) and torch.equal(fo, unfused)


@pytest.mark.parametrize("C,H,W", [(96, 55, 55), (256, 27, 27), (32, 20, 23)])
def test_lrn_maxpool_special_values_bitwise(device, C, H, W):
    """Signed zeros (Caffe's ReLU writes -0 for negative inputs), +-Inf, NaN
    and exact ties: the fused kernel's v_max3 windows (and their in-order
    re-walk when the maximum is zero) give the unfused strict-">" pooling's
    bits, sign of zero and NaN payload positions included."""
    import torch
    from rramsim import ops
    g = torch.Generator().manual_seed(23)
    N = 2
    x = 4 * torch.randn(N, C, H, W, generator=g)
    r = torch.rand(N, C, H, W, generator=g)
    x = torch.where(x < 0, x * 0.0, x)                       # ReLU's -0
    x = torch.where(r < 0.05, torch.zeros_like(x), x)        # +0 among the -0
    x[:, 3] = -0.0                                           # whole planes of zeros
    x[:, 4] = 0.0
    x[:, 5] = torch.where(r[:, 5] < 0.5, -0.0, 0.0)
    x.view(-1)[::4099] = float("inf")
    x.view(-1)[7::5003] = -float("inf")
    x.view(-1)[11::6007] = float("nan")
    x[:, 6] = 2.5                                            # exact ties everywhere
    x = x.to(device)
    alpha, beta, kk = 1e-4, 0.75, 1.0
    lrn = torch.empty_like(x)
    ops.lrn_fwd(x, lrn, None, N, C, H, W, 5, alpha, beta, kk)
    PH, PW = -(-(H - 3) // 2) + 1, -(-(W - 3) // 2) + 1
    unfused = torch.empty((N, C, PH, PW), device=device)
    ops.pool_fwd(lrn, unfused, None, (N, C, H, W, PH, PW, 3, 3, 2, 2, 0, 0), 0)
    fused = torch.full_like(unfused, 7.0)
    ops.lrn_maxpool_fwd(x, fused, N, C, H, W, PH, PW, 3, 2, 0, 5, alpha, beta, kk)
    fo = torch.full_like(unfused, 7.0)
    yo = torch.zeros(unfused.numel() * 6, dtype=torch.uint8, device=device)
    ops.lrn_maxpool_fwd_octets(x, fo, yo, N, C, H, W, PH, PW, 3, 2, 0, 5, alpha, beta, kk)
    torch.cuda.synchronize()
    ub = unfused.cpu().view(torch.int32)
    assert bool(torch.isnan(lrn).any()), "no NaN in the LRN planes"  # Inf inputs: Inf * Inf^-beta
    assert bool((ub == -2**31).any()), "no -0 maximum in the case"
    assert torch.equal(fused.cpu().view(torch.int32), ub)
    assert torch.equal(fo.cpu().view(torch.int32), ub)


def test_lrn_maxpool_fusion_in_alexnet_test_net(device):
    """Net folds norm1/norm2 into pool1/pool2 in the TEST phase; the net outputs
    are bit-identical to the unfused net."""
    import torch
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    outs = []
    for fuse in (False, True):
        caffe.set_random_seed(1701)
        net = caffe.Net(models.alexnet(test_batch=4), "test", models.net_options("alexnet", fuse_lrn_pool=fuse))
        net.forward()
        torch.cuda.synchronize()
        outs.append({b: net.blob(b).detach().cpu().clone() for b in ("pool1", "pool2", "fc8")})
        net.close()
    for b in ("pool1", "pool2", "fc8"):
        assert torch.equal(outs[0][b], outs[1][b]), b


@pytest.mark.parametrize("shape,k,s,p,method", [
    ((8, 32, 32, 32), 3, 2, 0, 0),      # CIFAR pool1: LDS-plane kernel, 3x3 MAX
    ((4, 20, 24, 24), 2, 2, 0, 0),      # LeNet-shaped 2x2 MAX
    ((3, 5, 13, 11), 3, 2, 1, 1),       # AVE (plane kernel, generic window)
    ((2, 3, 130, 130), 3, 2, 0, 0),     # planes > 16384: k_pool_max_fixed<3>
    ((2, 3, 130, 130), 5, 3, 1, 1),     # planes > 16384, AVE: k_pool_fwd
])
@pytest.mark.parametrize("slope", [0.0, 0.1])
def test_pool_relu_fused_equals_unfused(device, shape, k, s, p, method, slope):
    """rram_pool_relu_fwd == rram_pool_fwd then rram_relu_fwd in place, bit
    for bit (values incl. -0, +-Inf, NaN; the MAX argmax mask unchanged)."""
    import torch
    from rramsim import ops
    torch.manual_seed(11)
    x = torch.randn(*shape, device=device)
    x[0, 0, :4, :4] = -0.0
    x[0, 1, :2, :2] = float("-inf")
    x[-1, -1, 1, 1] = float("nan")
    x[-1, 0, :3, :3] = float("inf")
    N, C, H, W = shape
    PH = -(-(H + 2 * p - k) // s) + 1
    PW = -(-(W + 2 * p - k) // s) + 1
    if p and (PH - 1) * s >= H + p:
        PH -= 1
    if p and (PW - 1) * s >= W + p:
        PW -= 1
    geom = (N, C, H, W, PH, PW, k, k, s, s, p, p)
    yu = torch.empty((N, C, PH, PW), device=device)
    yf = torch.full_like(yu, 7.0)
    mu = torch.empty(yu.shape, dtype=torch.int32, device=device)
    mf = torch.full_like(mu, -7)
    ops.pool_fwd(x, yu, mu if method == 0 else None, geom, method)
    ops.relu_fwd(yu, yu, slope)
    ops.pool_relu_fwd(x, yf, mf if method == 0 else None, geom, method, slope)
    assert torch.equal(yu.view(torch.int32), yf.view(torch.int32))
    if method == 0:
        assert torch.equal(mu, mf)


@pytest.mark.parametrize("shape,k,s,p,method", [
    ((8, 32, 32, 32), 3, 2, 0, 0),      # MAX 3x3/2
    ((4, 32, 16, 16), 3, 2, 0, 1),      # CIFAR-10 full pool2: AVE 3x3/2
    ((3, 5, 13, 11), 3, 2, 1, 1),       # AVE, padded
])
@pytest.mark.parametrize("slope", [0.0, 0.1])
def test_pool_relu_bwd_fused_equals_unfused(device, shape, k, s, p, method, slope):
    """rram_pool_relu_bwd == rram_pool_bwd then rram_relu_bwd in place (the
    ReLU's output y = the pool's bottom data), bit for bit, incl. y = +-0 / NaN."""
    import torch
    from rramsim import ops
    torch.manual_seed(12)
    x = torch.randn(*shape, device=device)
    y = torch.where(x > 0, x, x * slope)            # the in-place ReLU's output
    y[0, 0, :2, :2] = -0.0
    y[-1, -1, 0, 0] = float("nan")
    N, C, H, W = shape
    PH = -(-(H + 2 * p - k) // s) + 1
    PW = -(-(W + 2 * p - k) // s) + 1
    if p and (PH - 1) * s >= H + p:
        PH -= 1
    if p and (PW - 1) * s >= W + p:
        PW -= 1
    geom = (N, C, H, W, PH, PW, k, k, s, s, p, p)
    top = torch.empty((N, C, PH, PW), device=device)
    mask = torch.empty(top.shape, dtype=torch.int32, device=device)
    ops.pool_fwd(y, top, mask if method == 0 else None, geom, method)
    dy = torch.randn_like(top)
    du, df = torch.empty_like(x), torch.full_like(x, 7.0)
    ops.pool_bwd(dy, mask if method == 0 else None, du, geom, method)
    ops.relu_bwd(y, du, du, slope)
    ops.pool_relu_bwd(dy, mask if method == 0 else None, df, geom, method, y, slope)
    assert torch.equal(du.view(torch.int32), df.view(torch.int32))


@pytest.mark.parametrize("slope", [0.0, 0.1])
def test_lrn_within_relu_bwd_fused_equals_unfused(device, slope):
    """rram_lrn_within_relu_bwd == rram_lrn_within_bwd then rram_relu_bwd in
    place (x = the ReLU's output = the LRN's bottom), bit for bit; CIFAR-10
    full norm1's parameters (local_size 3, WITHIN_CHANNEL)."""
    import torch
    from rramsim import ops
    torch.manual_seed(13)
    N, C, H, W = 4, 32, 16, 16
    x0 = 3 * torch.randn(N, C, H, W, device=device)
    x = torch.where(x0 > 0, x0, x0 * slope)
    x[0, 0, :2, :2] = -0.0
    alpha, beta = 5e-5, 0.75
    y, sc = torch.empty_like(x), torch.empty_like(x)
    ops.lrn_within_fwd(x, y, sc, N, C, H, W, 3, alpha, beta)
    dy = torch.randn_like(x)
    du, df = torch.empty_like(x), torch.full_like(x, 7.0)
    ops.lrn_within_bwd(x, sc, dy, du, N, C, H, W, 3, alpha, beta)
    ops.relu_bwd(x, du, du, slope)
    ops.lrn_within_relu_bwd(x, sc, dy, df, N, C, H, W, 3, alpha, beta, slope)
    assert torch.equal(du.view(torch.int32), df.view(torch.int32))


@pytest.mark.parametrize("net_name,phase", [("cifar10_quick", "test"), ("cifar10_full", "train")])
def test_pool_relu_fold_in_net(device, net_name, phase):
    """Net folds the in-place ReLU after a Pooling layer (CIFAR-10 pool1 ->
    relu1) into the pool's store, and (TRAIN) the backward of an in-place ReLU
    before a Pooling or LRN layer (relu2 -> pool2, relu3 -> pool3, relu1 ->
    norm1) into that layer's backward: blobs, loss and every parameter
    gradient equal to the net with the folds off."""
    import torch
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    outs = []
    for fuse in (False, True):
        caffe.set_random_seed(1701)
        spec = getattr(models, net_name)(train_batch=16, test_batch=16)
        net = caffe.Net(spec, phase, models.net_options(net_name, fuse_relu=fuse))
        net.forward()
        if phase == "train":
            net.backward()
        torch.cuda.synchronize()
        d = {b: net.blob(b).detach().cpu().clone() for b in ("pool1", "conv2")}
        if phase == "train":
            d.update({f"p{i}": q["diff"].detach().cpu().clone() for i, q in enumerate(net.params())})
        outs.append(d)
        net.close()
    # pool1 (this fold) bit for bit; the rest by value: the Conv / IP epilogue
    # ReLU fold (on with fuse_relu, relu2 / relu3 here) stores +0 where the
    # ReLU layer's v * 0 stores -0 for a negative v
    assert torch.equal(outs[0]["pool1"].view(torch.int32), outs[1]["pool1"].view(torch.int32))
    for b in outs[0]:
        assert torch.equal(outs[0][b], outs[1][b]), b


@pytest.mark.parametrize("size", [3, 5])
def test_lrn_within_fwd_bwd_vs_autograd(device, size):
    """cifar10_full's norm1/norm2 (lrn_layer.cpp WithinChannelForward/Backward)."""
    import torch
    from rramsim import ops
    torch.manual_seed(5)
    x = (3 * torch.randn(2, 4, 9, 8, device=device)).requires_grad_(True)
    alpha, beta = 5e-2, 0.75
    ref = _lrn_within_ref(x, size, alpha, beta)
    dy = torch.randn_like(ref)
    ref.backward(dy)
    N, C, H, W = x.shape
    y, sc, dx = torch.empty_like(ref), torch.empty_like(ref), torch.empty_like(ref)
    ops.lrn_within_fwd(x.detach(), y, sc, N, C, H, W, size, alpha, beta)
    ops.lrn_within_bwd(x.detach(), sc, dy, dx, N, C, H, W, size, alpha, beta)
    torch.testing.assert_close(y, ref.detach(), rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(dx, x.grad, rtol=1e-4, atol=1e-5)


def test_lrn_within_matches_numpy_oracle(device, oracle_mod):
    import torch
    from rramsim import ops
    rng = np.random.default_rng(9)
    x = rng.standard_normal((2, 3, 8, 8)).astype(np.float32) * 2
    ref = oracle_mod.lrn_within(x, 3, 5e-5 * 9, 0.75)
    y = torch.empty(x.shape, device=device)
    ops.lrn_within_fwd(_t(x, device), y, None, 2, 3, 8, 8, 3, 5e-5 * 9, 0.75)
    np.testing.assert_allclose(y.cpu().numpy(), ref, rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize("outer,C,inner,ignore,lw", [(100, 10, 1, -1, 1.0), (64, 10, 1, 3, 1.0),
                                                     (7, 5, 9, -1, 0.5), (3, 1000, 1, 2, 2.0)])
def test_softmax_loss_fused_fwd_bwd_equals_separate(device, outer, C, inner, ignore, lw):
    """rram_softmax_loss_fwd_bwd (the TRAIN-phase head in one launch) gives
    the loss and dx of rram_softmax_loss_fwd + rram_softmax_loss_bwd bit for
    bit, with and without an ignore label and a loss weight."""
    import torch
    from rramsim import ops
    torch.manual_seed(14)
    prob = torch.softmax(torch.randn(outer, C, inner, device=device), dim=1).contiguous()
    label = torch.randint(0, C, (outer, inner), device=device).float()
    l1, l2 = torch.zeros(1, device=device), torch.full((1,), 7.0, device=device)
    d1, d2 = torch.empty_like(prob), torch.full_like(prob, 7.0)
    ops.softmax_loss_fwd(prob, label, l1, outer, C, inner, ignore)
    ops.softmax_loss_bwd(prob, label, d1, outer, C, inner, ignore, lw)
    ops.softmax_loss_fwd_bwd(prob, label, l2, d2, outer, C, inner, ignore, lw)
    assert torch.equal(l1.view(torch.int32), l2.view(torch.int32))
    assert torch.equal(d1.view(torch.int32), d2.view(torch.int32))


@pytest.mark.parametrize("inner", [1, 6])
def test_softmax_loss_fwd_bwd_vs_autograd(device, inner):
    import torch
    import torch.nn.functional as F
    from rramsim import ops
    torch.manual_seed(6)
    outer, C = 17, 10
    logits = torch.randn(outer, C, inner, device=device).requires_grad_(True)
    label = torch.randint(0, C, (outer, inner), device=device)
    loss = F.cross_entropy(logits, label)
    loss.backward()
    prob = torch.empty(outer, C, inner, device=device)
    ops.softmax_fwd(logits.detach(), prob, outer, C, inner)
    out = torch.zeros(1, device=device)
    dx = torch.empty_like(prob)
    lf = label.float()
    ops.softmax_loss_fwd(prob, lf, out, outer, C, inner)
    ops.softmax_loss_bwd(prob, lf, dx, outer, C, inner)
    torch.testing.assert_close(out[0], loss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dx, logits.grad, rtol=1e-5, atol=1e-7)


def test_dropout_fwd_bwd(device):
    import torch
    from rramsim import ops
    x = torch.randn(1 << 16, device=device)
    dy = torch.randn_like(x)
    y, dx = torch.empty_like(x), torch.empty_like(x)
    mask = torch.empty(x.shape, dtype=torch.int32, device=device)
    ops.dropout_fwd(x, y, mask, 0.5, seed=11, layer_id=3, it=2)
    ops.dropout_bwd(dy, mask, dx, 0.5)
    keep = mask.bool()
    assert abs(keep.float().mean().item() - 0.5) < 0.01        # 64k draws, sd 0.002
    assert torch.equal(y, torch.where(keep, x * 2.0, torch.zeros_like(x)))
    assert torch.equal(dx, torch.where(keep, dy * 2.0, torch.zeros_like(x)))
    y2 = torch.empty_like(x)
    mask2 = torch.empty_like(mask)
    ops.dropout_fwd(x, y2, mask2, 0.5, seed=11, layer_id=3, it=2)
    assert torch.equal(mask, mask2)                             # counter-based: deterministic
    ops.dropout_fwd(x, y2, mask2, 0.5, seed=11, layer_id=3, it=3)
    assert not torch.equal(mask, mask2)                         # fresh mask per iteration


def test_concat_fwd_bwd(device):
    import torch
    from rramsim import ops
    a = torch.randn(3, 4, 5, device=device)
    b = torch.randn(3, 6, 5, device=device)
    dst = torch.empty(3, 10, 5, device=device)
    ops.concat_copy(a, dst, 3, 4 * 5, 10 * 5, 0)
    ops.concat_copy(b, dst, 3, 6 * 5, 10 * 5, 4 * 5)
    assert torch.equal(dst, torch.cat([a, b], 1))
    da, db = torch.empty_like(a), torch.empty_like(b)
    ops.concat_copy(da, dst, 3, 4 * 5, 10 * 5, 0, backward=True)
    ops.concat_copy(db, dst, 3, 6 * 5, 10 * 5, 4 * 5, backward=True)
    assert torch.equal(da, a) and torch.equal(db, b)


@pytest.mark.parametrize("xs,cout,k,s,p,g", [
    ((3, 64, 14, 14), 48, 1, 1, 0, 1),       # 1x1 (fp32 MFMA GEMM)
    ((3, 96, 14, 14), 208, 3, 1, 1, 1),      # 3x3, channel-octet kernel
    ((3, 16, 14, 14), 48, 5, 1, 2, 1),       # 5x5, channel-octet kernel (one K-tile)
    ((3, 24, 14, 14), 64, 3, 1, 1, 1),       # Cin % 16 != 0: patch kernel
    ((2, 3, 64, 64), 64, 7, 2, 3, 1),        # 7x7 stride 2 (GoogLeNet conv1, 64-bit tap mask)
    ((2, 3, 227, 227), 96, 11, 4, 0, 1),     # AlexNet conv1 (persistent ring kernel)
    ((2, 64, 13, 13), 128, 3, 1, 1, 2),      # groups
])
def test_conv_fwd_strided_equals_dense(device, xs, cout, k, s, p, g):
    """rram_conv2d_fwd_strided (the TEST-phase Concat fold's write): the
    output lands in a channel slice of a wider NCHW tensor, bit-identical to
    rram_conv2d_fwd, and nothing outside the slice is touched."""
    import torch
    from rramsim import ops
    rng = np.random.default_rng(31)
    x = torch.from_numpy(rng.standard_normal(xs).astype(np.float32)).to(device)
    w = torch.from_numpy((rng.standard_normal((cout, xs[1] // g, k, k)) * 0.05).astype(np.float32)).to(device)
    b = torch.from_numpy(rng.standard_normal(cout).astype(np.float32)).to(device)
    d = ops.conv_desc(xs, cout, k, s, p, 1, g)
    ref = torch.empty((xs[0], cout, d.out_h, d.out_w), device=device)
    ops.conv2d_fwd(d, x, w, b, ref, relu=True)
    ctot, off = cout + 40, 24
    big = torch.full((xs[0], ctot, d.out_h, d.out_w), float("nan"), device=device)
    ops.conv2d_fwd_strided(d, x, w, b, big[:, off:], ctot * d.out_h * d.out_w, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(big[:, off:off + cout], ref)
    assert torch.isnan(big[:, :off]).all() and torch.isnan(big[:, off + cout:]).all()


def test_concat_fold_in_googlenet_test_net(device):
    """Net folds the inception branch convolutions into their Concat tops in
    the TEST phase (each writes its channel slice; the Concat copies nothing):
    every Concat top and the net outputs are bit-identical to the unfolded net."""
    import torch
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    outs = []
    for fuse in (False, True):
        caffe.set_random_seed(1701)
        net = caffe.Net(models.googlenet(test_batch=4), "test", models.net_options("googlenet", fuse_concat=fuse))
        net.forward()
        torch.cuda.synchronize()
        names = [n for n in net.blob_names() if n.endswith("/output")] + ["loss3/classifier", "loss1/classifier"]
        outs.append({n: net.blob(n).detach().cpu().clone() for n in names})
        net.close()
    assert len(outs[0]) == 11
    for n in outs[0]:
        assert torch.equal(outs[0][n], outs[1][n]), n


def test_folded_blobs_materialise_when_read(device):
    """A blob a TEST-phase fold leaves unwritten (an inception branch output
    written straight into its Concat top; an LRN top computed inside the
    following MAX pool) holds its layer's output once the C-ABI hands it out
    (Net::materialize_blob): equal to the unfolded net's blob
    bit for bit, right away and after a further forward, and the net's
    outputs stay bit-identical."""
    import torch
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    cases = [("googlenet", models.googlenet, ["inception_3a/1x1", "inception_4e/pool_proj"], "fuse_concat",
              ["inception_3a/output", "loss3/classifier"]),
             ("alexnet", models.alexnet, ["norm1", "norm2"], "fuse_lrn_pool", ["pool2", "fc8"])]
    for name, build, folded, opt, outs in cases:
        got = {}
        for fuse in (False, True):
            caffe.set_random_seed(1701)
            net = caffe.Net(build(test_batch=4), "test", models.net_options(name, **{opt: fuse}))
            net.forward()
            torch.cuda.synchronize()
            first = {n: net.blob(n).detach().cpu().clone() for n in folded}
            net.forward()
            torch.cuda.synchronize()
            again = {n: net.blob(n).detach().cpu().clone() for n in folded + outs}
            got[fuse] = (first, again)
            net.close()
        for n in folded:
            assert torch.equal(got[True][0][n], got[False][0][n]), (name, n)
        for n in folded + outs:
            assert torch.equal(got[True][1][n], got[False][1][n]), (name, n)


def test_pooled_output_fold_materialises(device):
    """AlexNet TEST net, LRN + max pool folds on: from the second forward on,
    pool1 / pool2 (each read only by a convolution that takes their octet
    companion) are left unwritten in fp32 -- the kernel writes only the
    companion -- and are materialised when the C-ABI hands them out: bit for
    bit the unfused net's blobs; the net outputs stay bit-identical, and
    after the read the pool writes its fp32 output again."""
    import torch
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    got = {}
    for fuse in (False, True):
        caffe.set_random_seed(1701)
        net = caffe.Net(models.alexnet(test_batch=8), "test", models.net_options("alexnet", fuse_lrn_pool=fuse))
        for _ in range(3):
            net.forward()
        torch.cuda.synchronize()
        stale = {n: net.blob_stale(n) for n in ("pool1", "pool2", "norm1", "fc8")}
        got[fuse] = {n: net.blob(n).detach().cpu().clone() for n in ("pool1", "pool2", "fc8")}
        after = {n: net.blob_stale(n) for n in ("pool1", "pool2")}
        net.forward()
        torch.cuda.synchronize()
        again = {n: net.blob_stale(n) for n in ("pool1", "pool2")}
        net.close()
        if fuse:
            assert stale["pool1"] and stale["pool2"] and not stale["fc8"], stale
            assert not any(after.values()) and not any(again.values()), (after, again)
        else:
            assert not any(stale.values()), stale
    for n in got[False]:
        assert torch.equal(got[True][n], got[False][n]), n


def test_conv_output_fold_materialises(device):
    """AlexNet TEST net (round 6): conv3 and conv4, each read only by the next
    convolution through its octet companion, are left unwritten in fp32 --
    the channel-octet epilogue writes only the companion -- and materialised
    when the C-ABI hands them out: bit for bit the blobs of the same net with
    the fold off (fuse_conv_y: false); conv5 (read by pool5) is always
    written, the outputs are bit-identical, and after the read the producers
    write their fp32 outputs again."""
    import torch
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    got = {}
    names = ("conv3", "conv4", "conv5", "fc8")
    for fold in (False, True):
        caffe.set_random_seed(1701)
        net = caffe.Net(models.alexnet(test_batch=8), "test", models.net_options("alexnet", fuse_conv_y=fold))
        for _ in range(3):
            net.forward()
        torch.cuda.synchronize()
        stale = {n: net.blob_stale(n) for n in names}
        got[fold] = {n: net.blob(n).detach().cpu().clone() for n in names}
        after = {n: net.blob_stale(n) for n in names}
        net.forward()
        torch.cuda.synchronize()
        again = {n: net.blob_stale(n) for n in names}
        got[fold]["fc8_again"] = net.blob("fc8").detach().cpu().clone()
        net.close()
        if fold:
            assert stale["conv3"] and stale["conv4"] and not stale["conv5"] and not stale["fc8"], stale
            assert not any(after.values()) and not any(again.values()), (after, again)
        else:
            assert not any(stale.values()), stale
    for n in got[False]:
        assert torch.equal(got[True][n], got[False][n]), n


def test_conv_octets_only_epilogue_bit_identical(device):
    """rram_conv2d_fwd_octets with y = NULL (the convolution-output fold)
    writes the same companion as with y, on the AlexNet conv3 / conv4
    shapes the fold takes; a shape the channel-octet epilogue does not take
    refuses y = NULL instead of computing without an output."""
    import torch
    from rramsim import ops, RramError
    rng = np.random.default_rng(5)
    for (n, cin, cout, g) in [(4, 256, 384, 1), (4, 384, 384, 2)]:
        d = ops.conv_desc((n, cin, 13, 13), cout, 3, 1, 1, 1, g)
        assert ops.conv_output_octets_only(d) == 1
        x = torch.from_numpy(rng.standard_normal((n, cin, 13, 13)).astype(np.float32)).to(device)
        w = torch.from_numpy((rng.standard_normal((cout, cin // g, 3, 3)) * 0.05).astype(np.float32)).to(device)
        b = torch.from_numpy(rng.standard_normal(cout).astype(np.float32)).to(device)
        y = torch.empty((n, cout, 13, 13), device=device)
        yo1 = torch.zeros(n * cout * 169 * 6, dtype=torch.uint8, device=device)
        yo2 = torch.full_like(yo1, 7)
        ops.conv2d_fwd_octets(d, x, None, w, b, y, yo1, relu=True)
        ops.conv2d_fwd_octets(d, x, None, w, b, None, yo2, relu=True)
        torch.cuda.synchronize()
        assert torch.equal(yo1, yo2)
    d = ops.conv_desc((2, 3, 32, 32), 32, 5, 1, 2, 1, 1)          # fp32-engine shape: no companion epilogue
    assert ops.conv_output_octets_only(d) == 0
    x = torch.randn(2, 3, 32, 32, device=device)
    w = torch.randn(32, 3, 5, 5, device=device)
    yo = torch.zeros(2 * 32 * 32 * 32 * 6, dtype=torch.uint8, device=device)
    with pytest.raises(RramError):
        ops.conv2d_fwd_octets(d, x, None, w, None, None, yo)


@pytest.mark.parametrize("n,cin,cout,hw", [(3, 64, 64, 56), (3, 192, 96, 28), (2, 480, 192, 14), (2, 832, 160, 7)])
def test_conv1x1_octets_only_epilogue_bit_identical(device, n, cin, cout, hw):
    """Round 6: the 1x1 kernels (register ring for M <= 64, LDS-DMA above)
    with y = NULL write the same companion as with y (GoogLeNet conv2 /
    3x3_reduce and inception reduce shapes)."""
    import torch
    from rramsim import ops
    rng = np.random.default_rng(9)
    d = ops.conv_desc((n, cin, hw, hw), cout, 1, 1, 0, 1, 1)
    assert ops.conv_output_octets_only(d) == 1
    x = torch.from_numpy(np.maximum(rng.standard_normal((n, cin, hw, hw)), 0).astype(np.float32)).to(device)
    w = torch.from_numpy((rng.standard_normal((cout, cin, 1, 1)) * 0.05).astype(np.float32)).to(device)
    b = torch.from_numpy(rng.standard_normal(cout).astype(np.float32)).to(device)
    y = torch.empty((n, cout, hw, hw), device=device)
    yo1 = torch.zeros(n * cout * hw * hw * 6, dtype=torch.uint8, device=device)
    yo2 = torch.full_like(yo1, 7)
    ops.conv2d_fwd_octets(d, x, None, w, b, y, yo1, relu=True)
    ops.conv2d_fwd_octets(d, x, None, w, b, None, yo2, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(yo1, yo2)


def test_conv1x1_output_fold_in_googlenet(device):
    """GoogLeNet TEST net (round 6): the 1x1 reductions read only by a 3x3 /
    5x5 convolution that takes their octet companion are left unwritten in
    fp32 after the first forwards and materialised when handed out -- bit
    for bit the blobs with the fold off; the loss outputs are bit-identical."""
    import torch
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    names = ["conv2/3x3_reduce"] + [f"inception_{b}/{k}_reduce" for b in ("3a", "3b", "4a", "4e", "5b")
                                     for k in ("3x3", "5x5")]
    outs = ["loss1/loss1", "loss2/loss1", "loss3/loss3", "loss3/classifier"]
    got, stale = {}, {}
    for fold in (False, True):
        caffe.set_random_seed(1701)
        net = caffe.Net(models.googlenet(test_batch=4), "test", models.net_options("googlenet", fuse_conv_y=fold))
        for _ in range(3):
            net.forward()
        torch.cuda.synchronize()
        stale[fold] = {n: net.blob_stale(n) for n in names}
        got[fold] = {n: net.blob(n).detach().cpu().clone() for n in names + outs}
        net.close()
    assert not any(stale[False].values()), stale[False]
    assert stale[True]["conv2/3x3_reduce"] and stale[True]["inception_3a/3x3_reduce"], stale[True]
    for n in names + outs:
        assert torch.equal(got[True][n], got[False][n]), n


def test_pooled_output_fold_needs_a_sole_convolution_reader(device):
    """A second reader of pool1 (here a ReLU writing its own top) keeps the
    pool writing its fp32 top: pool1 is never stale, the extra reader sees
    the unfused values, and pool2 (still read by conv3 alone) stays folded."""
    import torch
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    proto = models.alexnet(test_batch=4) + (
        '\nlayer { name: "pool1_relu" type: "ReLU" bottom: "pool1" top: "pool1_relu" }\n')
    got = {}
    for fuse in (False, True):
        caffe.set_random_seed(1701)
        net = caffe.Net(proto, "test", models.net_options("alexnet", fuse_lrn_pool=fuse))
        for _ in range(3):
            net.forward()
        torch.cuda.synchronize()
        stale = (net.blob_stale("pool1"), net.blob_stale("pool2"))
        got[fuse] = {n: net.blob(n).detach().cpu().clone() for n in ("pool1", "pool1_relu", "pool2", "fc8")}
        net.close()
        if fuse:
            assert stale == (False, True), stale
    for n in got[False]:
        assert torch.equal(got[True][n], got[False][n]), n


@pytest.mark.parametrize("shape,k,s,p", [((2, 5, 13, 11), 3, 2, 0), ((3, 4, 32, 32), 3, 2, 0), ((2, 3, 16, 16), 3, 2, 1),
                                         ((1, 2, 64, 64), 2, 2, 0), ((1, 1, 70, 70), 3, 2, 0)])
def test_max_pool_bwd_bit_exact(device, shape, k, s, p):
    """MAX pooling backward (pooling_layer.cu:145-167: each input element
    sums, in (a, b) row-major order, the gradients of the pooled outputs whose
    argmax it is) bit for bit against a float32 numpy restatement, on the
    plane-per-block kernel (H * W <= 4096) and the per-element one (70 x 70)."""
    import torch
    from rramsim import ops
    torch.manual_seed(21)
    N, C, H, W = shape
    PH = -(-(H + 2 * p - k) // s) + 1
    PW = -(-(W + 2 * p - k) // s) + 1
    if p > 0:
        PH -= (PH - 1) * s >= H + p
        PW -= (PW - 1) * s >= W + p
    x = torch.randn(shape, device=device)
    geom = (N, C, H, W, PH, PW, k, k, s, s, p, p)
    y = torch.empty((N, C, PH, PW), device=device)
    mask = torch.empty((N, C, PH, PW), dtype=torch.int32, device=device)
    ops.pool_fwd(x, y, mask, geom, 0)
    dy = torch.randn_like(y)
    dx = torch.empty_like(x)
    ops.pool_bwd(dy, mask, dx, geom, 0)
    m, g = mask.cpu().numpy(), dy.cpu().numpy()
    ref = np.zeros(shape, np.float32)
    for n in range(N):
        for c in range(C):
            for h in range(H):
                for w in range(W):
                    phs = 0 if h + p < k else (h + p - k) // s + 1
                    phe = min((h + p) // s + 1, PH)
                    pws = 0 if w + p < k else (w + p - k) // s + 1
                    pwe = min((w + p) // s + 1, PW)
                    acc = np.float32(0)
                    for a in range(phs, phe):
                        for b in range(pws, pwe):
                            if m[n, c, a, b] == h * W + w:
                                acc = np.float32(acc + g[n, c, a, b])
                    ref[n, c, h, w] = acc
    assert np.array_equal(dx.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_ip_rows_chain_bit_identical(device):
    """The packed-row chain of two InnerProducts on the bf16x6 engine
    (rram_ip_fwd_rows, fc6 -> fc7 at b256): the first layer's split-K reduce
    writes its output and the second layer's packed input; the second reads
    that instead of packing -- both outputs bit-identical to rram_ip_fwd
    (bias, ReLU, the split-K order); an AlexNet TEST forward's fc7 equals
    rram_ip_fwd over its fc6 blob."""
    import torch
    from rramsim import caffe, models, ops
    torch.manual_seed(3)
    M, K1, N1, N2 = 256, 9216, 4096, 4096
    x = torch.randn(M, K1, device=device)
    w1 = torch.randn(N1, K1, device=device) * 0.01
    b1 = torch.randn(N1, device=device)
    w2 = torch.randn(N2, N1, device=device) * 0.01
    b2 = torch.randn(N2, device=device)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=device)
    wsb = ws.numel()
    nb, bmc = ops.ip_rows_pack_bytes(M, N2, N1, wsb)
    assert nb > 0 and bmc > 0
    rows = torch.empty(nb, dtype=torch.uint8, device=device)
    y1 = torch.empty(M, N1, device=device)
    assert ops.ip_fwd_rows(x, None, w1, b1, y1, rows, bmc, M, N1, K1, relu=True, workspace=ws)
    y2 = torch.empty(M, N2, device=device)
    assert not ops.ip_fwd_rows(y1, rows, w2, b2, y2, None, 0, M, N2, N1, relu=True, workspace=ws)
    r1 = torch.empty_like(y1)
    ops.ip_fwd(x, w1, b1, r1, M, N1, K1, relu=True, workspace=ws)
    r2 = torch.empty_like(y2)
    ops.ip_fwd(r1, w2, b2, r2, M, N2, N1, relu=True, workspace=ws)
    torch.cuda.synchronize()
    assert torch.equal(y1.view(torch.int32), r1.view(torch.int32))
    assert torch.equal(y2.view(torch.int32), r2.view(torch.int32))
    # the net: fc7 (read through fc6's packed rows) == rram_ip_fwd over the fc6 blob
    caffe.set_stream_from_torch()
    caffe.set_random_seed(1701)
    net = caffe.Net(models.alexnet(test_batch=256), "test", models.net_options("alexnet"))
    net.forward()
    fc6 = net.blob("fc6").detach().clone()
    fc7 = net.blob("fc7").detach().clone()
    ps = net.params()
    w7, b7 = ps[12]["data"], ps[13]["data"]
    assert w7.numel() == 4096 * 4096 and b7.numel() == 4096
    ref = torch.empty_like(fc7)
    ops.ip_fwd(fc6, w7, b7, ref, 256, 4096, 4096, relu=True, workspace=ws)
    torch.cuda.synchronize()
    assert torch.equal(fc7.view(torch.int32), ref.view(torch.int32))
    # pool5 == rram_pool_fwd
    # over conv5, and fc6 == rram_ip_fwd over pool5
    conv5 = net.blob("conv5").detach().clone()
    pool5 = net.blob("pool5").detach().clone()
    rp = torch.empty_like(pool5)
    from rramsim import _kernels as KK
    ops.pool_fwd(conv5, rp, None, (256, 256, 13, 13, 6, 6, 3, 3, 2, 2, 0, 0), KK.RRAM_POOL_MAX)
    w6, b6 = ps[10]["data"], ps[11]["data"]
    r6 = torch.empty_like(fc6)
    ops.ip_fwd(pool5, w6, b6, r6, 256, 4096, 9216, relu=True, workspace=ws)
    torch.cuda.synchronize()
    assert torch.equal(pool5.view(torch.int32), rp.view(torch.int32))
    assert torch.equal(fc6.view(torch.int32), r6.view(torch.int32))
    net.close()
