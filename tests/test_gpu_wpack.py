"""Packed-weight companions (include/rram_kernels.h rram_conv2d_fwd_cached):
the bf16x6 engine's pre-split fragment form of a convolution's weights, kept
next to the weight blob (SyncedMemory::wpack) while the weights are unchanged,
so the Monte-Carlo driver splits map-invariant convolution weights once
instead of once per map.  No reference counterpart (the reference re-reads w
through cuBLAS each call, conv_layer.cu:7-25); the gates are bit-identity:
a cached forward equals rram_conv2d_fwd bit for bit, and a whole MC map's
convolutions equal plain forwards of the net's own blobs with the weights the
map ran on — including the conv-fault extension, where every map rewrites the
convolution weights and a stale pack would show."""
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


CASES = [
    dict(x=(2, 3, 227, 227), cout=96, k=11, s=4, p=0, g=1),   # AlexNet conv1: persistent conv1 kernel
    dict(x=(2, 96, 27, 27), cout=256, k=5, s=1, p=2, g=2),    # conv2: channel-octet kernel
    dict(x=(2, 256, 13, 13), cout=384, k=3, s=1, p=1, g=1),   # conv3: channel-octet kernel
    dict(x=(2, 24, 20, 20), cout=96, k=3, s=1, p=1, g=1),     # Cin % 16 != 0: patch kernel
    dict(x=(3, 480, 14, 14), cout=192, k=1, s=1, p=0, g=1),   # 1x1: k_conv1x1_x6 (16-byte loads)
    dict(x=(3, 832, 7, 7), cout=48, k=1, s=1, p=0, g=1),      # 1x1: k_conv1x1_x6 (4-byte loads)
]


@pytest.mark.parametrize("cs", CASES)
def test_cached_pack_bit_identical(device, cs):
    import torch
    from rramsim import ops
    rng = np.random.default_rng(5)
    x = rng.standard_normal(cs["x"]).astype(np.float32)
    cg = cs["x"][1] // cs["g"]
    w = (rng.standard_normal((cs["cout"], cg, cs["k"], cs["k"])) * 0.05).astype(np.float32)
    w2 = (rng.standard_normal(w.shape) * 0.05).astype(np.float32)
    b = rng.standard_normal(cs["cout"]).astype(np.float32)
    d = ops.conv_desc(cs["x"], cs["cout"], cs["k"], cs["s"], cs["p"], 1, cs["g"])
    assert ops.f32_engine_for_conv(d) == ops.ENGINE_BF16X6
    nb = ops.conv_weight_pack_bytes(d)
    assert nb > 0
    xd, wd, w2d, bd = T(x, device), T(w, device), T(w2, device), T(b, device)
    ys = (cs["x"][0], cs["cout"], d.out_h, d.out_w)
    ref, ref2 = torch.empty(ys, device=device), torch.empty(ys, device=device)
    ops.conv2d_fwd(d, xd, wd, bd, ref, relu=True)
    ops.conv2d_fwd(d, xd, w2d, bd, ref2, relu=True)
    wp = torch.zeros(nb, dtype=torch.uint8, device=device)
    for valid, wt, want in ((False, wd, ref), (True, wd, ref),
                            (True, w2d, ref),      # the pack, not w, is read: still w's result
                            (False, w2d, ref2)):   # repacked from w2
        y = torch.full(ys, float("nan"), device=device)
        ops.conv2d_fwd_cached(d, xd, None, wt, wp, valid, bd, y, relu=True)
        np.testing.assert_array_equal(N(y), N(want), err_msg=f"valid={valid}")


def test_no_pack_for_fp32_engine_shapes(device):
    """Shapes the fp32 MFMA engine takes (1x1 with C % 16 != 0, 7x7 stride 2)
    have no pack; the cached entry point refuses a pack for them instead of
    ignoring it.  (A 1x1 with C % 16 == 0 runs k_conv1x1_x6 and has one.)"""
    import torch
    from rramsim import ops
    from rramsim import _kernels as K
    assert ops.conv_weight_pack_bytes(ops.conv_desc((2, 32, 14, 14), 64, 1, 1, 0, 1, 1)) == 2 * 2 * 3072
    for xs, co, k, s, p in (((2, 24, 14, 14), 64, 1, 1, 0), ((2, 3, 64, 64), 64, 7, 2, 3)):
        d = ops.conv_desc(xs, co, k, s, p, 1, 1)
        assert ops.conv_weight_pack_bytes(d) == 0
        x = torch.zeros(xs, device=device)
        w = torch.zeros((co, xs[1], k, k), device=device)
        y = torch.empty((xs[0], co, d.out_h, d.out_w), device=device)
        wp = torch.zeros(1024, dtype=torch.uint8, device=device)
        with pytest.raises(K.RramError):
            ops.conv2d_fwd_cached(d, x, None, w, wp, False, None, y)


def _conv_outputs_match(net, device, geo):
    import torch
    from rramsim import ops
    ps = net.params()
    k, p = 0, {}
    for name, typ, npar in net.layers():
        if npar:
            p[name] = [ps[k + j]["data"] for j in range(npar)]
            k += npar
    for name, (bot, cout, kk, st, pad, g) in geo.items():
        xb = net.blob(bot)
        xs = tuple(int(v) for v in xb.shape)
        d = ops.conv_desc(xs, cout, kk, st, pad, 1, g)
        y = torch.empty((xs[0], cout, d.out_h, d.out_w), device=device)
        ops.conv2d_fwd(d, xb.contiguous().view(xs), p[name][0].contiguous(), p[name][1].contiguous(), y, relu=True)
        np.testing.assert_array_equal(N(net.blob(name)).reshape(N(y).shape), N(y), err_msg=name)


ALEX = {"conv1": ("data", 96, 11, 4, 0, 1), "conv2": ("pool1", 256, 5, 1, 2, 2),
        "conv3": ("pool2", 384, 3, 1, 1, 1), "conv4": ("conv3", 384, 3, 1, 1, 2),
        "conv5": ("conv4", 256, 3, 1, 1, 2)}


@pytest.mark.parametrize("conv_faults", [False, True])
def test_mc_maps_with_cached_packs(device, conv_faults):
    """AlexNet b16, three MC maps with the packs kept across maps: the last
    map's conv1-5 outputs equal plain forwards with the weights that map ran
    on.  Reference semantics (IP faults only) reuse every pack; with the
    conv-fault extension each map's injection invalidates them."""
    from rramsim import caffe, make_inject_cfg, models
    caffe.set_stream_from_torch()
    caffe.set_random_seed(11)
    opts = models.net_options("alexnet")
    if conv_faults:
        opts["fault_layers"] = "InnerProduct,Convolution"
    net = caffe.Net(models.alexnet(test_batch=16), "test", opts)
    mc = caffe.MonteCarlo(net, make_inject_cfg(0.05), seed=3, max_maps=8)
    for m in range(3):
        mc.run(m, 1)
    _conv_outputs_match(net, device, ALEX)
    mc.close()
    net.close()


def test_mc_overlapped_injection_equals_serial(device, monkeypatch):
    """RRAM_MC_OVERLAP=1 (the injection on a side stream after conv2, under
    the rest of the layers before the first faultable one; off by default)
    gives the serial order's per-map accuracy / loss and final logits bit
    for bit, and so does the graph replay with it set (serial)."""
    from rramsim import caffe, make_inject_cfg, models
    caffe.set_stream_from_torch()
    res = []
    for ov in ("0", "1", "graph"):
        monkeypatch.setenv("RRAM_MC_OVERLAP", "1" if ov == "graph" else ov)
        caffe.set_random_seed(13)
        net = caffe.Net(models.alexnet(test_batch=16), "test", models.net_options("alexnet"))
        mc = caffe.MonteCarlo(net, make_inject_cfg(0.02), seed=5, max_maps=8)
        if ov == "graph":
            mc.set_graph(True)
        mc.run(0, 3)
        if ov == "graph":
            assert mc.graph_active()
        st = mc.stats()
        res.append((st["per_map"], st["broken"], N(net.blob("fc8"))))
        mc.close()
        net.close()
    for r in res[1:]:
        assert res[0][0] == r[0] and res[0][1] == r[1]
        np.testing.assert_array_equal(res[0][2], r[2])


@pytest.mark.parametrize("conv_faults", [False, True])
def test_mc_prefix_reuse_bit_identical(device, conv_faults):
    """MonteCarlo prefix reuse (include/rram_caffe.h rram_mc_set_reuse_prefix,
    an opt-in workload): maps that start at the first faultable layer give the
    full forward's per-map accuracy / loss, broken-cell counts and final logits
    bit for bit; with the conv-fault extension the prefix is the data layer
    alone and the option changes nothing."""
    from rramsim import caffe, make_inject_cfg, models
    caffe.set_stream_from_torch()
    res = []
    for reuse in (False, True):
        caffe.set_random_seed(17)
        opts = models.net_options("alexnet")
        if conv_faults:
            opts["fault_layers"] = "InnerProduct,Convolution"
        net = caffe.Net(models.alexnet(test_batch=16), "test", opts)
        mc = caffe.MonteCarlo(net, make_inject_cfg(0.03), seed=9, max_maps=8)
        if reuse:
            mc.set_reuse_prefix(True)
        mc.run(0, 4)
        st = mc.stats()
        res.append((st["per_map"], st["broken"], N(net.blob("fc8")), N(net.blob("pool5"))))
        mc.close()
        net.close()
    for r in res[1:]:
        assert res[0][0] == r[0] and res[0][1] == r[1]
        np.testing.assert_array_equal(res[0][2], r[2])
    np.testing.assert_array_equal(res[0][3], res[1][3])


def test_net_input_octet_companion_not_stale(device):
    """A convolution reading a net input packs the input's octet companion
    itself.  The Input blob's data pointer was handed out (rram_net_blob), so
    a caller can write the next batch through it with no mutable access: the
    second forward must convolve the new batch, not the companion of the old
    one (SyncedMemory::valid_octets refuses exposed memory)."""
    import torch
    from rramsim import caffe, ops
    shape, cout = (2, 32, 13, 13), 96
    d = ops.conv_desc(shape, cout, 3, 1, 1, 1, 1)
    assert ops.conv_input_octets(d) == 1                 # this convolution reads the companion
    txt = ('layer { name: "x" type: "Input" top: "x" input_param { shape { dim: 2 dim: 32 dim: 13 dim: 13 } } }\n'
           'layer { name: "conv" type: "Convolution" bottom: "x" top: "y" convolution_param { num_output: 96 '
           'kernel_size: 3 pad: 1 weight_filler { type: "gaussian" std: 0.1 } bias_filler { type: "constant" value: 0.5 } } }\n')
    caffe.set_stream_from_torch()
    net = caffe.Net(txt, "test")
    xb = net.blob("x")                                    # kept across both batches
    p = net.params()
    w, b = p[0]["data"].view(cout, 32, 3, 3), p[1]["data"]
    rng = np.random.default_rng(3)
    for batch in range(3):
        x = torch.from_numpy(rng.standard_normal(shape).astype(np.float32)).to(device)
        xb.copy_(x)
        net.forward()
        ref = torch.empty((2, cout, 13, 13), device=device)
        ops.conv2d_fwd(d, x, w, b, ref)
        np.testing.assert_array_equal(N(net.blob("y")), N(ref), err_msg=f"batch {batch}")
    net.close()


def test_shared_weights_different_geometry_under_mc(device):
    """Two convolutions share one weight blob (param names) but differ in pad,
    so their packed weights follow different tile plans; with the packs kept
    across MC maps (SyncedMemory::wpack), each must keep its own key (the
    whole descriptor) and both outputs equal plain forwards."""
    from rramsim import caffe, make_inject_cfg, ops
    txt = ('layer { name: "x" type: "DummyData" top: "x" dummy_data_param { shape { dim: 4 dim: 32 dim: 15 dim: 15 } '
           'data_filler { type: "gaussian" std: 1 } } }\n'
           'layer { name: "ca" type: "Convolution" bottom: "x" top: "ya" param { name: "w" } param { name: "b" } '
           'convolution_param { num_output: 64 kernel_size: 3 pad: 1 weight_filler { type: "gaussian" std: 0.1 } '
           'bias_filler { type: "constant" value: 0.1 } } }\n'
           'layer { name: "cb" type: "Convolution" bottom: "x" top: "yb" param { name: "w" } param { name: "b" } '
           'convolution_param { num_output: 64 kernel_size: 3 pad: 0 weight_filler { type: "gaussian" std: 0.1 } '
           'bias_filler { type: "constant" value: 0.1 } } }\n'
           'layer { name: "fc" type: "InnerProduct" bottom: "yb" top: "fc" inner_product_param { num_output: 10 '
           'weight_filler { type: "gaussian" std: 0.01 } } }\n')
    caffe.set_stream_from_torch()
    caffe.set_random_seed(21)
    net = caffe.Net(txt, "test")
    mc = caffe.MonteCarlo(net, make_inject_cfg(0.05), seed=2, max_maps=4)
    for m in range(3):
        mc.run(m, 1)
    import torch
    ps = net.params()
    w, b = ps[0]["data"].view(64, 32, 3, 3), ps[1]["data"]
    x = net.blob("x").contiguous()
    for name, pad in (("ya", 1), ("yb", 0)):
        d = ops.conv_desc((4, 32, 15, 15), 64, 3, 1, pad, 1, 1)
        y = torch.empty((4, 64, d.out_h, d.out_w), device=device)
        ops.conv2d_fwd(d, x, w, b, y)
        np.testing.assert_array_equal(N(net.blob(name)).reshape(N(y).shape), N(y), err_msg=name)
    mc.close()
    net.close()
