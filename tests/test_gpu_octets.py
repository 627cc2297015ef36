"""Channel-octet companions (include/rram_kernels.h rram_conv2d_fwd_octets):
the pre-split bf16x3 form of an activation that a producer (the bf16x6
convolution's epilogue, the fused LRN + max-pool) writes next to its fp32
output so the next convolution skips its input pack.  No reference
counterpart (an inference-time layout of this build); the gates are
bit-identity: the companion equals the exact split of the fp32 tensor
(numpy restatement below), and every fp32 output is bit-identical with and
without companions, down to a whole AlexNet forward."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def N(t):
    import torch
    torch.cuda.synchronize()
    return t.detach().cpu().numpy().copy()


def T(a, device):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def _bf16_rne(x):
    """float32 -> bf16 bits, round to nearest even (finite inputs)."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def _f32(b):
    return (b.astype(np.uint32) << 16).view(np.float32)


def octets_ref(x):
    """[n][C][H][W] fp32 -> [n][C/8][H][W][3][8] bf16 bits: x = xh + xm + xl."""
    x = x.astype(np.float32)
    h = _bf16_rne(x)
    r1 = (x - _f32(h)).astype(np.float32)
    m = _bf16_rne(r1)
    r2 = (r1 - _f32(m)).astype(np.float32)
    lo = _bf16_rne(r2)
    n, c, hh, ww = x.shape
    out = np.stack([t.reshape(n, c // 8, 8, hh, ww).transpose(0, 1, 3, 4, 2) for t in (h, m, lo)], axis=4)
    return np.ascontiguousarray(out)


def _oct_buf(shape, device):
    import torch
    return torch.zeros(int(np.prod(shape)) * 6, dtype=torch.uint8, device=device)


def _as_u16(t, shape):
    n, c, h, w = shape
    return N(t).view(np.uint16).reshape(n, c // 8, h, w, 3, 8)


def test_octet_split_is_exact():
    """The three terms sum back to x exactly (numpy restatement)."""
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((2, 16, 3, 5)) * np.exp(rng.uniform(-20, 20, (2, 16, 3, 5)))).astype(np.float32)
    o = octets_ref(x).astype(np.uint16)
    s = (_f32(o[..., 0, :]).astype(np.float64) + _f32(o[..., 1, :]) + _f32(o[..., 2, :]))
    back = s.transpose(0, 1, 4, 2, 3).reshape(x.shape)
    np.testing.assert_array_equal(back.astype(np.float32), x)


@pytest.mark.parametrize("shape", [(3, 16, 7, 9), (2, 24, 13, 13), (1, 8, 1, 1)])
def test_pack_octets_bit_exact(device, shape):
    from rramsim import ops
    rng = np.random.default_rng(11)
    x = rng.standard_normal(shape).astype(np.float32)
    o = _oct_buf(shape, device)
    ops.pack_octets(T(x, device), o, *shape)
    np.testing.assert_array_equal(_as_u16(o, shape), octets_ref(x))


# (x shape, cout, k, pad, group): channel-octet kernel shapes (AlexNet conv2-5
# per-group forms) and shapes on the other kernels (companion packed afterwards)
OCT_CASES = [
    dict(x=(3, 96, 27, 27), cout=256, k=5, p=2, g=2),
    dict(x=(3, 256, 13, 13), cout=384, k=3, p=1, g=1),
    dict(x=(3, 384, 13, 13), cout=384, k=3, p=1, g=2),
    dict(x=(3, 384, 13, 13), cout=256, k=3, p=1, g=2),
    dict(x=(2, 32, 14, 14), cout=64, k=1, p=0, g=1),     # 1x1: register-ring kernel, companion from its epilogue
    dict(x=(3, 192, 28, 28), cout=96, k=1, p=0, g=1),    # 1x1: LDS-DMA kernel, companion from its epilogue
    dict(x=(2, 64, 7, 7), cout=48, k=1, p=0, g=1),       # 1x1: 4-byte loads, partial last column tile
    dict(x=(2, 16, 9, 9), cout=40, k=1, p=0, g=1),       # 1x1: a row block with one octet of rows
    dict(x=(2, 16, 20, 20), cout=32, k=3, p=1, g=1),     # M = 32: patch / fp32 path
]


@pytest.mark.parametrize("cs", OCT_CASES)
@pytest.mark.parametrize("relu", [False, True])
def test_conv_octets_bit_identical(device, cs, relu):
    """rram_conv2d_fwd_octets: y bit-identical to rram_conv2d_fwd with and
    without an input companion; the output companion bit-identical to the
    split of y."""
    import torch
    from rramsim import ops
    rng = np.random.default_rng(21)
    x = rng.standard_normal(cs["x"]).astype(np.float32)
    cg = cs["x"][1] // cs["g"]
    w = (rng.standard_normal((cs["cout"], cg, cs["k"], cs["k"])) * 0.05).astype(np.float32)
    b = rng.standard_normal(cs["cout"]).astype(np.float32)
    d = ops.conv_desc(cs["x"], cs["cout"], cs["k"], 1, cs["p"], 1, cs["g"])
    yshape = (cs["x"][0], cs["cout"], d.out_h, d.out_w)
    xd, wd, bd = T(x, device), T(w, device), T(b, device)
    y0 = torch.empty(yshape, device=device)
    ops.conv2d_fwd(d, xd, wd, bd, y0, relu=relu)
    xo = _oct_buf(cs["x"], device)
    ops.pack_octets(xd, xo, *cs["x"])
    for use_xo in (False, True):
        y1 = torch.full(yshape, float("nan"), device=device)
        yo = _oct_buf(yshape, device)
        ops.conv2d_fwd_octets(d, xd, xo if use_xo else None, wd, bd, y1, yo, relu=relu)
        ref = N(y0)
        np.testing.assert_array_equal(N(y1), ref)
        np.testing.assert_array_equal(_as_u16(yo, yshape), octets_ref(ref))


def test_lrn_maxpool_octets_bit_identical(device):
    """rram_lrn_maxpool_fwd_octets: y bit-identical to rram_lrn_maxpool_fwd,
    the companion bit-identical to the split of y (AlexNet norm1 / pool1 and
    norm2 / pool2 geometry)."""
    import torch
    from rramsim import ops
    rng = np.random.default_rng(31)
    for (n, c, h, w) in [(3, 96, 55, 55), (3, 256, 27, 27)]:
        x = np.abs(rng.standard_normal((n, c, h, w))).astype(np.float32) * 50
        ph = pw = int(np.ceil((h - 3) / 2)) + 1
        xd = T(x, device)
        y0 = torch.empty((n, c, ph, pw), device=device)
        ops.lrn_maxpool_fwd(xd, y0, n, c, h, w, ph, pw, 3, 2, 0, 5, 1e-4, 0.75)
        y1 = torch.full((n, c, ph, pw), float("nan"), device=device)
        yo = _oct_buf((n, c, ph, pw), device)
        ops.lrn_maxpool_fwd_octets(xd, y1, yo, n, c, h, w, ph, pw, 3, 2, 0, 5, 1e-4, 0.75)
        ref = N(y0)
        np.testing.assert_array_equal(N(y1), ref)
        np.testing.assert_array_equal(_as_u16(yo, (n, c, ph, pw)), octets_ref(ref))
        # y = NULL (the pooled-output fold): the same companion, no fp32 store
        yo2 = _oct_buf((n, c, ph, pw), device)
        ops.lrn_maxpool_fwd_octets(xd, None, yo2, n, c, h, w, ph, pw, 3, 2, 0, 5, 1e-4, 0.75)
        np.testing.assert_array_equal(_as_u16(yo2, (n, c, ph, pw)), octets_ref(ref))


def test_alexnet_forward_pool_companions_only_bit_identical(device):
    """A whole AlexNet TEST forward where only pool1 / pool2 hand their
    companions to conv2 / conv3 and conv4 / conv5 pack their inputs
    (RRAM_OCTETS=2, read once per process, so it runs in a child): every
    convolution's output equals a plain rram_conv2d_fwd of the net's own
    bottom blob bit for bit."""
    import os
    import subprocess
    import sys
    if os.environ.get("RRAM_OCTETS") == "2":
        _alexnet_check(device)
        return
    env = dict(os.environ, RRAM_OCTETS="2")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "gpu",
                        __file__ + "::test_alexnet_forward_pool_companions_only_bit_identical"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_alexnet_forward_bit_identical(device):
    """The same check with the default (RRAM_OCTETS=1: pool1 / pool2 / conv3 /
    conv4 all hand their companions to conv2-5)."""
    _alexnet_check(device)


def _alexnet_check(device):
    import torch
    from rramsim import caffe, models, ops
    caffe.set_stream_from_torch()
    caffe.set_random_seed(7)
    B = 16
    net = caffe.Net(models.alexnet(test_batch=B), "test", models.net_options("alexnet"))
    net.forward()
    net.forward()  # the first forward after setup already uses companions; run two to cover reuse
    ps = net.params()
    k, p = 0, {}
    for name, typ, npar in net.layers():
        if npar:
            p[name] = [ps[k + j]["data"] for j in range(npar)]
            k += npar
    geo = {"conv2": ("pool1", 256, 5, 2, 2), "conv3": ("pool2", 384, 3, 1, 1),
           "conv4": ("conv3", 384, 3, 1, 2), "conv5": ("conv4", 256, 3, 1, 2)}
    used = 0
    for name, (bot, cout, kk, pad, g) in geo.items():
        xb = net.blob(bot)
        xs = tuple(int(v) for v in xb.shape)
        d = ops.conv_desc(xs, cout, kk, 1, pad, 1, g)
        used += ops.conv_input_octets(d)
        y = torch.empty((xs[0], cout, d.out_h, d.out_w), device=device)
        ops.conv2d_fwd(d, xb.contiguous().view(xs), p[name][0].contiguous(), p[name][1].contiguous(), y, relu=True)
        np.testing.assert_array_equal(N(net.blob(name)).reshape(N(y).shape), N(y), err_msg=name)
    assert used == 4  # all four convolutions take the companion path at this batch
