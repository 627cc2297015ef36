"""fp32-level accuracy guard for every bf16x6 kernel at the grids the
headline bench launches (AlexNet b256, one Monte-Carlo fault map).

The per-layer parity checks (tests/_ref64.py) bound every output by
1e-4 · Σ|a·b|, the north_star tolerance; that bound would also pass a kernel
that had silently lost fp32 accuracy (a bf16x3 split errs by ~2^-16 of
Σ|a·b|).  This guard is the fp32 bar, per kernel the bench runs:

  k_conv1_ring_x6  conv1 (3x227x227, 96 x 11 x 11, stride 4)
  k_conv_cb_x6     conv2 (5x5, g2), conv3, conv4 (g2), conv5 (g2)
  k_gemm_x6        fc6 (256 x 4096 x 9216), fc7 (256 x 4096 x 4096)

On the bench's own activations and (faulted) weights — one MC map of the
bench's net, every layer's bottom blob read back — the layer is evaluated on
the bf16x6 engine and on the fp32-MFMA engine (v_mfma_f32_32x32x2_f32, plain
fp32 products) at b256, and both are compared with a float64 evaluation
(images sampled across the batch for the convolutions, all 256 rows for the
IP layers).  In units of the element's Σ|a·b| + |bias|:

  max err(bf16x6)  <= 1e-6                      (fp32 level; the gate is 1e-4)
  max err(bf16x6)  <= 2 x max err(fp32 MFMA)
  mean err(bf16x6) <= 2 x mean err(fp32 MFMA)   (the tight bound: a dropped
                                                  2^-16 product term raises it ~8x)

tests/test_x6_guard_emulation.py shows on the CPU that these bounds reject
each single dropped product term of the split and the bf16x3 form, and
profiles/r04_fp32_guard.txt records a GPU build with one term dropped
(RRAM_X6_DROP) failing this file.  The net's fused-ReLU outputs are also
checked to equal relu() of the ops-level bf16x6 outputs bit for bit, so the
kernel measured here is the one the bench's layers run.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BATCH = 256
# images sampled for the float64 convolutions: both ends, around the middle,
# and neighbours (tiles of some kernels span image boundaries)
SAMPLE = [0, 1, 2, 63, 64, 127, 128, 129, 191, 200, 253, 254, 255]
CONVS = {"conv1": ("data", 96, 11, 4, 0, 1), "conv2": ("pool1", 256, 5, 1, 2, 2),
         "conv3": ("pool2", 384, 3, 1, 1, 1), "conv4": ("conv3", 384, 3, 1, 1, 2),
         "conv5": ("conv4", 256, 3, 1, 1, 2)}
IPS = {"fc6": ("pool5", 4096), "fc7": ("fc6", 4096)}


def N(t):
    import torch
    torch.cuda.synchronize()
    return t.detach().cpu().numpy().copy()


@pytest.fixture(scope="module")
def bench_map(device):
    """One MC map of the bench's net (models.alexnet b256, p_fault 0.01, the
    bench's seed): per layer the bottom blob, weights, bias and the net's own
    (fused-ReLU) output, copied to the device as plain tensors."""
    import torch
    from rramsim import caffe, make_inject_cfg, models
    caffe.set_stream_from_torch()
    caffe.set_random_seed(1701)
    net = caffe.Net(models.alexnet(test_batch=BATCH), "test", models.net_options("alexnet"))
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
    for name, (bot, *_r) in list(CONVS.items()) + list(IPS.items()):
        out[name] = dict(x=net.blob(bot).clone(), w=par[name][0], b=par[name][1], y=net.blob(name).clone())
    torch.cuda.synchronize()
    mc.close()
    net.close()
    return out


def _engines(run):
    """run(engine) -> device tensor; both engines' outputs, engine restored."""
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


@pytest.mark.parametrize("name", list(CONVS))
def test_conv_bf16x6_fp32_level_at_bench_grid(device, bench_map, name):
    import torch
    from rramsim import ops
    from _ref64 import conv64
    bot, cout, k, s, p, g = CONVS[name]
    L = bench_map[name]
    x, w, b = L["x"], L["w"], L["b"]
    d = ops.conv_desc(tuple(x.shape), cout, k, s, p, 1, g)
    assert d.num == BATCH
    wv = w.view(cout, x.shape[1] // g, k, k)

    def run(eng):
        assert ops.f32_engine_for_conv(d) == eng       # the shape really runs on that engine
        y = torch.empty((BATCH, cout, d.out_h, d.out_w), device=device)
        ops.conv2d_fwd(d, x, wv, b, y, relu=False)
        return y

    got = _engines(run)
    # the bench's layer (fused ReLU, octet companions, cached packs) is this kernel
    assert torch.equal(L["y"].view(BATCH, cout, d.out_h, d.out_w), torch.relu(got[ops.ENGINE_BF16X6]))
    xs = N(x)[SAMPLE]
    ref, scale = conv64(xs, N(wv), N(b), s, p, g)
    _judge(name, {e: N(y)[SAMPLE] for e, y in got.items()}, ref, scale)


@pytest.mark.parametrize("name", list(IPS))
def test_ip_bf16x6_fp32_level_at_bench_grid(device, bench_map, name):
    import torch
    from rramsim import ops
    from _ref64 import ip64
    bot, nout = IPS[name]
    L = bench_map[name]
    x, w, b = L["x"], L["w"], L["b"]
    K = x.numel() // BATCH
    ws = torch.empty((256 << 20) // 4, device=device)      # the layer's workspace bound

    def run(eng):
        assert ops.f32_engine_for_ip(BATCH, nout, K) == eng
        y = torch.empty((BATCH, nout), device=device)
        ops.ip_fwd(x, w, b, y, BATCH, nout, K, relu=False, workspace=ws)
        return y

    got = _engines(run)
    assert torch.equal(L["y"].view(BATCH, nout), torch.relu(got[ops.ENGINE_BF16X6]))
    ref, scale = ip64(N(x).reshape(BATCH, K), N(w).reshape(nout, K), N(b))
    _judge(name, {e: N(y) for e, y in got.items()}, ref, scale)
