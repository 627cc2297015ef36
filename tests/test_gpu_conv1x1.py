"""k_conv1x1_x6: the 1 x 1 convolution (GoogLeNet's inception 1x1 / reduce /
pool_proj layers, conv_layer.cu:9-30 with kernel 1) on the bf16x6 engine.

  * shape sweep: both load widths (16-byte for H*W % 4 == 0, 4-byte for the
    7 x 7 layers), every tile configuration the plan picks (M from 16 to 384,
    rows not a multiple of 32, an odd number of 16-channel K-tiles, tiles
    spanning images, partial last tiles), bias + fused ReLU, against float64
    (the north_star 1e-4 scaled gate) and the fp32-level guard against the
    fp32-MFMA engine on the same data (tests/_ref64.py);
  * the Concat-fold write (image stride) is bit-identical to the dense one;
  * at the C5 grid (GoogLeNet b256, one MC fault map): the net's own 1x1
    layers equal relu() of this kernel bit for bit, and pass the fp32 guard.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def N(t):
    import torch
    torch.cuda.synchronize()
    return t.detach().cpu().numpy().copy()


def _engines(run):
    from rramsim import ops
    prev = ops.get_f32_engine()
    try:
        res = {}
        for eng in (ops.ENGINE_F32, ops.ENGINE_BF16X6):
            ops.set_f32_engine(eng)
            res[eng] = run(eng)
        return res
    finally:
        ops.set_f32_engine(prev)


def _judge(name, got, ref, scale):
    from rramsim import ops
    from _ref64 import x6_guard_failures
    err = {}
    for eng, y in got.items():
        r = np.abs(y.astype(np.float64) - ref) / np.maximum(scale, 1e-300)
        err[eng] = (float(r.max()), float(r.mean()))
    f32, x6 = err[ops.ENGINE_F32], err[ops.ENGINE_BF16X6]
    print(f"{name}: err / sum|a*b|  max  f32 {f32[0]:.3e} bf16x6 {x6[0]:.3e}   "
          f"mean  f32 {f32[1]:.3e} bf16x6 {x6[1]:.3e}")
    bad = x6_guard_failures(x6, f32)
    assert not bad, f"{name}: bf16x6 " + "; ".join(bad)


SHAPES = [
    ((2, 192, 28, 28), 64),     # inception_3a/1x1
    ((2, 192, 28, 28), 96),     # 3x3_reduce
    ((2, 192, 28, 28), 16),     # 5x5_reduce (one 32-row block, half padded)
    ((1, 64, 56, 56), 64),      # conv2/3x3_reduce
    ((3, 480, 14, 14), 192),    # inception_4a/1x1 (tiles span images)
    ((3, 528, 14, 14), 160),    # inception_4e: 33 K-tiles of 16 channels
    ((4, 832, 7, 7), 384),      # inception_5b/1x1: 4-byte loads, 128-row tiles
    ((2, 512, 4, 4), 128),      # loss1/conv
    ((5, 32, 9, 9), 24),        # 4-byte loads, M % 8 != 0
    ((2, 16, 10, 10), 300),     # many row tiles, M tail
    ((7, 48, 12, 12), 112),     # 1008 positions: partial last column tile
]


@pytest.mark.parametrize("xs,cout", SHAPES)
def test_conv1x1_x6_vs_float64_and_fp32_guard(device, xs, cout):
    import torch
    from rramsim import ops
    from _ref64 import assert_scaled, conv64
    rng = np.random.default_rng(sum(xs) + cout)
    x = torch.from_numpy(rng.standard_normal(xs).astype(np.float32)).to(device)
    w = torch.from_numpy((rng.standard_normal((cout, xs[1], 1, 1)) / np.sqrt(xs[1])).astype(np.float32)).to(device)
    b = torch.from_numpy(rng.standard_normal(cout).astype(np.float32)).to(device)
    d = ops.conv_desc(xs, cout, 1, 1, 0, 1, 1)

    def run(eng):
        assert ops.f32_engine_for_conv(d) == eng
        y = torch.empty((xs[0], cout, xs[2], xs[3]), device=device)
        ops.conv2d_fwd(d, x, w, b, y, relu=False)
        return y

    got = _engines(run)
    yr = torch.empty_like(got[ops.ENGINE_BF16X6])
    ops.conv2d_fwd(d, x, w, b, yr, relu=True)
    assert torch.equal(yr, torch.relu(got[ops.ENGINE_BF16X6]))
    ref, scale = conv64(N(x), N(w), N(b))
    assert_scaled(N(got[ops.ENGINE_BF16X6]), ref, scale, f"1x1 {xs}->{cout}")
    _judge(f"1x1 {xs}->{cout}", {e: N(y) for e, y in got.items()}, ref, scale)


@pytest.mark.parametrize("xs,cout", [((3, 480, 14, 14), 192), ((4, 832, 7, 7), 128), ((2, 192, 28, 28), 16)])
def test_conv1x1_x6_strided_equals_dense(device, xs, cout):
    import torch
    from rramsim import ops
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.standard_normal(xs).astype(np.float32)).to(device)
    w = torch.from_numpy((rng.standard_normal((cout, xs[1], 1, 1)) * 0.05).astype(np.float32)).to(device)
    b = torch.from_numpy(rng.standard_normal(cout).astype(np.float32)).to(device)
    d = ops.conv_desc(xs, cout, 1, 1, 0, 1, 1)
    assert ops.f32_engine_for_conv(d) == ops.ENGINE_BF16X6
    ref = torch.empty((xs[0], cout, xs[2], xs[3]), device=device)
    ops.conv2d_fwd(d, x, w, b, ref, relu=True)
    ctot, off = cout + 40, 24
    big = torch.full((xs[0], ctot, xs[2], xs[3]), float("nan"), device=device)
    ops.conv2d_fwd_strided(d, x, w, b, big[:, off:], ctot * xs[2] * xs[3], relu=True)
    torch.cuda.synchronize()
    assert torch.equal(big[:, off:off + cout], ref)
    assert torch.isnan(big[:, :off]).all() and torch.isnan(big[:, off + cout:]).all()


# C5 grid: (layer, bottom blob, (concat top, channel offset) or None when the
# layer's own top is materialised)
GN = {
    "inception_3a/1x1": ("pool2/3x3_s2", ("inception_3a/output", 0)),
    "inception_3a/3x3_reduce": ("pool2/3x3_s2", None),
    "inception_4a/1x1": ("pool3/3x3_s2", ("inception_4a/output", 0)),
    "inception_4e/5x5_reduce": ("inception_4d/output", None),
    "inception_5b/1x1": ("inception_5a/output", ("inception_5b/output", 0)),
    "loss1/conv": ("loss1/ave_pool", None),
}
SAMPLE = [0, 1, 2, 127, 128, 254, 255]


@pytest.fixture(scope="module")
def gn_map(device):
    import torch
    from rramsim import caffe, make_inject_cfg, models
    caffe.set_stream_from_torch()
    caffe.set_random_seed(1701)
    net = caffe.Net(models.googlenet(test_batch=256), "test", models.net_options("googlenet"))
    mc = caffe.MonteCarlo(net, make_inject_cfg(0.01), seed=1701, max_maps=4)
    mc.run(0, 1)
    torch.cuda.synchronize()
    ps = net.params()
    k, par = 0, {}
    for name, typ, npar in net.layers():
        if npar:
            par[name] = [ps[k + j]["data"].clone() for j in range(npar)]
            k += npar
    out = {}
    for name, (bot, top) in GN.items():
        w, b = par[name]
        if top is None:
            y = net.blob(name).clone()
        else:
            cc = b.numel()
            y = net.blob(top[0])[:, top[1]:top[1] + cc].clone()
        out[name] = dict(x=net.blob(bot).clone(), w=w, b=b, y=y)
    torch.cuda.synchronize()
    mc.close()
    net.close()
    return out


@pytest.mark.parametrize("name", list(GN))
def test_googlenet_1x1_at_c5_grid(device, gn_map, name):
    import torch
    from rramsim import ops
    from _ref64 import conv64
    L = gn_map[name]
    x, w, b = L["x"], L["w"], L["b"]
    cout = b.numel()
    d = ops.conv_desc(tuple(x.shape), cout, 1, 1, 0, 1, 1)
    wv = w.view(cout, x.shape[1], 1, 1)

    def run(eng):
        assert ops.f32_engine_for_conv(d) == eng
        y = torch.empty((x.shape[0], cout, x.shape[2], x.shape[3]), device=device)
        ops.conv2d_fwd(d, x, wv, b, y, relu=False)
        return y

    got = _engines(run)
    assert torch.equal(L["y"].reshape(got[ops.ENGINE_BF16X6].shape), torch.relu(got[ops.ENGINE_BF16X6]))
    ref, scale = conv64(N(x)[SAMPLE], N(wv), N(b))
    _judge(name, {e: N(y)[SAMPLE] for e, y in got.items()}, ref, scale)
