"""The five BASELINE.json configs as GPU parity tests (SURVEY.md §8 preamble).

C1 LeNet stuck-at           -> test_gpu_host.py (forward, solver Fail step, MC)
C2 CIFAR-10 quick, quantisation + lognormal variation, MC maps
C3 AlexNet b256 MC inference -> per-layer fp64 parity at the bench batch
C4 CIFAR-10 full fault-aware training (mean 5e6, std 1.5e6, prob 5, threshold;
   run_different_th.sh:3-10), unfused and fused, bit-exact vs the oracle tail
C5 GoogLeNet fault-rate sweep (p = 0.1 % and 10 %), per-layer SA0/SA1 ratios

Floating-point layer outputs are checked layer by layer on the GPU's own
bottom blobs against a float64 evaluation, within 1e-4 of Σ|a·b| (tests/_ref64.py);
fault decisions and stuck / quantised weights are bit-exact against the oracle.
"""
import math

import numpy as np
import pytest

import _ref64 as R

pytestmark = pytest.mark.gpu


def N(t):
    import torch
    torch.cuda.synchronize()
    return t.detach().cpu().numpy().copy()


@pytest.fixture(scope="module")
def rs(device):
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    caffe.set_random_seed(1701)
    return caffe, models


def _params_by_layer(net):
    ps = net.params()
    out, k = {}, 0
    for name, typ, npar in net.layers():
        if npar:
            out[name] = [N(ps[k + j]["data"]) for j in range(npar)]
            k += npar
    return out


def _oracle_cfg(oracle_mod, c):
    return oracle_mod.InjectCfg(c.thr_fault, c.thr_neg, c.thr_zero, c.thr_sa1, c.stuck_scale, c.g_max,
                                c.quant_levels, c.var_sigma, c.cell_mode, 0)


def _binom_ok(k, n, p, z=3.8):
    """test_random_number_generator.cpp:17-19 bound: |k/n - p| <= 3.8 sigma."""
    return abs(k / n - p) <= z * math.sqrt(max(p * (1 - p), 1e-300) / n) + 1.0 / n


# ----------------------------------------------------------------------- C2
def _quick_cfgs(net, sigma, p=0.01):
    from rramsim import make_inject_cfg
    cfgs = []
    for f in net.failure_params():
        gmax = float(f["data"].abs().max().item()) or 1.0
        cfgs.append(make_inject_cfg(p, 10, 20, 10, quant_levels=16, g_max=gmax, var_sigma=sigma, stuck_scale=gmax))
    return cfgs


@pytest.mark.parametrize("sigma", [0.0, 0.1])
def test_c2_cifar10_quick_quant_lognormal_map(rs, oracle_mod, sigma):
    """C2: one CIFAR-10 quick MC map with 16-level conductance quantisation,
    lognormal variation (sigma 0.1) and 1 % stuck-at on the 66,250 IP weights.
    Broken decisions and counts are exact; quantised / stuck weights are
    bit-exact (sigma = 0: every weight); the exp(sigma z) factor within 1e-5;
    the forward of the faulted net within 1e-4 of Σ|a·b| per layer."""
    caffe, models = rs
    B = 100
    net = caffe.Net(models.cifar10_quick(test_batch=B), "test", models.net_options("cifar10_quick"))
    fps = net.failure_params()
    assert sum(f["count"] for f in fps) == 66_250
    clean = [N(f["data"]) for f in fps]
    cfgs = _quick_cfgs(net, sigma)
    mc = caffe.MonteCarlo(net, cfgs, seed=1701, max_maps=8)
    mc.run(5, 1)
    st = mc.stats()
    for i, f in enumerate(fps):
        ref, nb = oracle_mod.inject(clean[i], _oracle_cfg(oracle_mod, cfgs[i]), 1701, 5, i)
        got = N(f["data"])
        assert st["broken"][i] == nb, (i, st["broken"][i], nb)
        same = got.view(np.uint32) == ref.view(np.uint32)
        if sigma == 0.0:
            assert same.all(), f"blob {i}: quantised/stuck weights differ at {np.flatnonzero(~same)[:8]}"
        else:
            s = cfgs[i].stuck_scale
            stuck = np.isin(ref, np.float32([-s, 0.0, s]))
            assert same[stuck].all()
            np.testing.assert_allclose(got[~same], ref[~same], rtol=1e-5, atol=0)
    # the faulted forward, layer by layer (cifar10_quick_train_test.prototxt)
    p = _params_by_layer(net)
    x = N(net.blob("data")).reshape(B, 3, 32, 32)
    R.check_conv(N(net.blob("conv1")), x, p["conv1"][0].reshape(32, 3, 5, 5), p["conv1"][1], 1, 2, what="conv1")
    R.check_conv(N(net.blob("conv2")), N(net.blob("pool1")), p["conv2"][0].reshape(32, 32, 5, 5), p["conv2"][1],
                 1, 2, relu=True, what="conv2")
    R.check_conv(N(net.blob("conv3")), N(net.blob("pool2")), p["conv3"][0].reshape(64, 32, 5, 5), p["conv3"][1],
                 1, 2, relu=True, what="conv3")
    R.check_ip(N(net.blob("ip1")), N(net.blob("pool3")), p["ip1"][0], p["ip1"][1], what="ip1")
    R.check_ip(N(net.blob("ip2")), N(net.blob("ip1")), p["ip2"][0], p["ip2"][1], what="ip2")
    # the map's accuracy record is the accuracy of these logits
    logits = N(net.blob("ip2")).reshape(B, 10)
    label = N(net.blob("label")).reshape(B)
    assert abs(st["per_map"][0][0] - oracle_mod.accuracy(logits, label) / B) < 1e-6
    mc.close()
    net.close()


def test_c2_cifar10_quick_fault_rate_binomial(rs):
    """C2 over 64 maps: the broken fraction of the 66,250 IP cells lies in the
    3.8 sigma binomial bound, every map differs, and map records are per map."""
    caffe, models = rs
    net = caffe.Net(models.cifar10_quick(test_batch=100), "test", models.net_options("cifar10_quick"))
    n = sum(f["count"] for f in net.failure_params())
    mc = caffe.MonteCarlo(net, _quick_cfgs(net, 0.1), seed=3, max_maps=64)
    mc.run(0, 64)
    st = mc.stats()
    assert st["maps"] == 64 and len(st["per_map"]) == 64
    assert _binom_ok(sum(st["broken"]), 64 * n, 0.01)
    sm = mc.summary()
    assert 0.0 <= sm["accuracy"]["mean"] <= 1.0 and sm["accuracy"]["maps"] == 64
    mc.close()
    net.close()


# ----------------------------------------------------------------------- C3
def test_c3_alexnet_b256_per_layer_fp64(rs, oracle_mod):
    """C3 at the bench's batch (256, so the split-K / tile choices are the
    bench's): every conv1-5 and fc6-8 output within 1e-4 of Σ|a·b| of a
    float64 evaluation on the GPU's own bottom blob (conv layers on 8 images
    spread over the batch, fc layers on all 256 rows), the LRN + max-pool fusion
    within 1e-5 relative, and one faulted map's fc6-8 likewise."""
    from rramsim import make_inject_cfg
    caffe, models = rs
    B = 256
    net = caffe.Net(models.alexnet(test_batch=B), "test", models.net_options("alexnet"))
    sel = np.array([0, 37, 64, 101, 128, 190, 222, 255])
    sh = {"conv1": ((96, 3, 11, 11), 4, 0, 1, "data"), "conv2": ((256, 48, 5, 5), 1, 2, 2, "pool1"),
          "conv3": ((384, 256, 3, 3), 1, 1, 1, "pool2"), "conv4": ((384, 192, 3, 3), 1, 1, 2, "conv3"),
          "conv5": ((256, 192, 3, 3), 1, 1, 2, "conv4")}

    def check_all(fc_only=False):
        p = _params_by_layer(net)
        worst = {}
        if not fc_only:
            for k, (wsh, s, pad, g, bot) in sh.items():
                x = N(net.blob(bot))[sel]
                worst[k] = R.check_conv(N(net.blob(k))[sel], x, p[k][0].reshape(wsh), p[k][1], s, pad, g,
                                        relu=True, what=k)
            for src, dst in (("conv1", "pool1"), ("conv2", "pool2")):
                ref = R.maxpool64(R.lrn64(N(net.blob(src))[sel], 5, 1e-4, 0.75), 3, 2)
                np.testing.assert_allclose(N(net.blob(dst))[sel], ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
        for k, bot, relu in (("fc6", "pool5", True), ("fc7", "fc6", True), ("fc8", "fc7", False)):
            worst[k] = R.check_ip(N(net.blob(k)), N(net.blob(bot)), p[k][0], p[k][1], relu=relu, what=k)
        return worst

    net.forward()
    worst = check_all()
    print("C3 clean worst err/scale:", {k: f"{v:.2e}" for k, v in worst.items()})
    # one faulted map (stuck-at 1 %, SA split 5/90/5): fc6-8 see the faulted weights
    mc = caffe.MonteCarlo(net, make_inject_cfg(0.01, 5, 90, 5), seed=1701, max_maps=2)
    mc.run(3, 1)
    fps = net.failure_params()
    assert sum(f["count"] for f in fps) == 58_631_144
    worst = check_all(fc_only=True)
    print("C3 map-3 worst err/scale:", {k: f"{v:.2e}" for k, v in worst.items()})
    n = sum(f["count"] for f in fps)
    assert _binom_ok(sum(mc.stats()["broken"]), n, 0.01)
    mc.close()
    net.close()


# ----------------------------------------------------------------------- C4
def _fault_index(net):
    """failure param k -> learnable param index (net.cpp:484-489 registry)."""
    ptr = {p["data"].data_ptr(): j for j, p in enumerate(net.params())}
    return [ptr[f["data"].data_ptr()] for f in net.failure_params()]


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("threshold", [1e-3, 1e-5])
def test_c4_cifar10_full_training_tail_bit_exact(rs, oracle_mod, fused, threshold):
    """C4: cifar10_full fault-aware training with the fork's solver settings
    (cifar10_full_solver.prototxt: lr 0.001, momentum 0.9, decay 0.004; ip1
    decay_mult 250) and run_different_th.sh's fault model (mean 5e6, std 1.5e6,
    prob 5 -> neg/zero/pos 5/90/5, threshold strategy).  The raw gradients are
    captured at on_gradients_ready (solver.cpp:296-298); the oracle then applies
    Regularize -> SGDUpdate -> threshold -> Update -> Fail (solver.cpp:300-305)
    and every weight, history and endurance value after 3 iterations equals the
    GPU's bit for bit, broken counts included, fused tail or not."""
    caffe, models = rs
    caffe.set_random_seed(2024)
    sp = models.solver(base_lr=0.001, momentum=0.9, weight_decay=0.004, max_iter=100, failure_mean=5e6,
                       failure_std=1.5e6, failure_prob=(5, 90, 5), threshold=threshold)
    s = caffe.Solver(sp, models.cifar10_full(train_batch=100, test_batch=100),
                     models.net_options("cifar10_full", fused_update=fused))
    net = s.net
    ps = net.params()
    fidx = _fault_index(net)
    assert sum(net.failure_params()[k]["count"] for k in range(len(fidx))) == 10_250
    fs = s.fail_state()
    w = [N(p["data"]) for p in ps]
    h = [np.zeros_like(x) for x in w]
    e = [N(a) for a, _ in fs]
    v = [N(b) for _, b in fs]
    # initial broken fraction: P(e <= 0) = Phi(-mean/std)
    from rramsim import gaussian_fault_rate
    n = sum(len(x) for x in e)
    assert _binom_ok(sum(int((x <= 0).sum()) for x in e), n, gaussian_fault_rate(5e6, 1.5e6))
    assert np.isin(np.concatenate(v), [-1.0, 0.0, 1.0]).all()
    grads = []
    s.set_gradient_callback(lambda: grads.append([N(p["diff"]) for p in ps]))
    f32 = np.float32
    for it in range(3):
        s.step(1)
        g = grads[-1]
        lr = f32(s.learning_rate())
        nb_total = []
        for j, p in enumerate(ps):
            k = fidx.index(j) if j in fidx else -1
            decay = f32(0.004) * f32(p["decay_mult"])
            local = lr * f32(p["lr_mult"])
            thr = f32(threshold) * (f32(p["lr_mult"]) * lr)          # strategy.cpp:13-14
            w[j], _, h[j], ek, nb = oracle_mod.fused_update_fail(
                w[j], g[j], h[j], e[k] if k >= 0 else None, v[k] if k >= 0 else None, decay, f32(0.9), local,
                k >= 0, thr if k >= 0 else 0.0)
            if k >= 0:
                e[k] = ek
                nb_total.append((k, nb))
            got = N(p["data"])
            assert np.array_equal(got.view(np.uint32), w[j].view(np.uint32)), (it, j)
        for k, nb in nb_total:
            assert np.array_equal(N(fs[k][0]).view(np.uint32), e[k].view(np.uint32)), (it, k)
            assert s.broken_counts()[k] == nb, (it, k)
    s.close()


# ----------------------------------------------------------------------- C5
@pytest.mark.parametrize("p_fault", [0.001, 0.1])
def test_c5_googlenet_sweep_point(rs, oracle_mod, p_fault):
    """C5: a GoogLeNet (train_val TEST, b32) map at fault rate p with per-layer
    SA ratios (aux heads 20/60/20, loss3 5/90/5).  Reference semantics fault
    only the InnerProduct blobs (net.cpp:484-489): each is bit-exact against
    the oracle's injection and its broken count exact; over 4 maps the broken
    fraction and the -1/0/+1 split of every weight blob pass the 3.8 sigma
    binomial bound; the IP layers' outputs within 1e-4 of Σ|a·b|."""
    _c5_sweep_point(rs, oracle_mod, p_fault, 32)


def test_c5_googlenet_b256_sweep_point(rs, oracle_mod):
    """C5 at the bench batch (b256, p = 2 %): the same gates on the kernels
    and grids the googlenet_sweep workload runs (per-layer fp64 checks on the
    first four images of the batch)."""
    _c5_sweep_point(rs, oracle_mod, 0.02, 256)


def _c5_sweep_point(rs, oracle_mod, p_fault, B):
    from rramsim import make_inject_cfg
    caffe, models = rs
    net = caffe.Net(models.googlenet(test_batch=B), "test", models.net_options("googlenet"))
    fps = net.failure_params()
    names = [n for n, t, k in net.layers() if t == "InnerProduct"]
    assert names == ["loss1/fc", "loss1/classifier", "loss2/fc", "loss2/classifier", "loss3/classifier"]
    assert len(fps) == 10 and fps[-2]["count"] == 1_024_000
    ratios = [(20, 60, 20)] * 8 + [(5, 90, 5)] * 2
    scale = 7.0                                       # stuck values -7 / 0 / +7 never collide with weights
    cfgs = [make_inject_cfg(p_fault, *r, stuck_scale=scale) for r in ratios]
    clean = [N(f["data"]) for f in fps]
    mc = caffe.MonteCarlo(net, cfgs, seed=99, max_maps=8)
    split = np.zeros((len(fps), 3), np.int64)
    broken = np.zeros(len(fps), np.int64)
    excluded = np.zeros(len(fps), np.int64)
    for m in range(4):
        mc.reset()
        mc.run(m, 1)
        st = mc.stats()
        for i, f in enumerate(fps):
            ref, nb = oracle_mod.inject(clean[i], _oracle_cfg(oracle_mod, cfgs[i]), 99, m, i)
            got = N(f["data"])
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (m, i)
            assert st["broken"][i] == nb, (m, i)
            broken[i] += nb
            if i % 2 == 0:                            # weights: count the stuck values of the cells
                keep = ~np.isin(clean[i], [-scale, 0.0, scale])   # whose clean value differs from all three
                excluded[i] = int((~keep).sum())
                g = got[keep]
                split[i] += [(g == -scale).sum(), (g == 0).sum(), (g == scale).sum()]
    for i, f in enumerate(fps):
        assert _binom_ok(int(broken[i]), 4 * f["count"], p_fault), (i, broken[i])
        if i % 2 == 0:
            nb_seen = int(split[i].sum())               # xavier can draw an exact 0.0: those cells are
            assert broken[i] - 4 * excluded[i] <= nb_seen <= broken[i]   # left out of the split count
            tot = sum(ratios[i])
            for c in range(3):
                if nb_seen >= 100:
                    assert _binom_ok(int(split[i][c]), nb_seen, ratios[i][c] / tot), (i, c, split[i])
    # the last map's faulted IP layers, per layer (fused ReLU on the two fc heads)
    p = _params_by_layer(net)
    for k, bot, relu in (("loss1/fc", "loss1/conv", True), ("loss1/classifier", "loss1/fc", False),
                         ("loss2/fc", "loss2/conv", True), ("loss2/classifier", "loss2/fc", False),
                         ("loss3/classifier", "pool5/7x7_s1", False)):
        R.check_ip(N(net.blob(k)), N(net.blob(bot)), p[k][0], p[k][1], relu=relu, what=k)
    # and convolutions of the trunk on the same forward; the inception
    # branches are read from their slices of the Concat top, which the
    # TEST-phase Concat fold has them write directly (rram_conv2d_fwd_strided)
    R.check_conv(N(net.blob("conv1/7x7_s2"))[:4], N(net.blob("data"))[:4], p["conv1/7x7_s2"][0].reshape(64, 3, 7, 7),
                 p["conv1/7x7_s2"][1], 2, 3, relu=True, what="conv1/7x7_s2")
    R.check_conv(N(net.blob("inception_4a/output"))[:4, 400:448], N(net.blob("inception_4a/5x5_reduce"))[:4],
                 p["inception_4a/5x5"][0].reshape(48, 16, 5, 5), p["inception_4a/5x5"][1], 1, 2, relu=True,
                 what="inception_4a/5x5")
    R.check_conv(N(net.blob("inception_3a/output"))[:4, 0:64], N(net.blob("pool2/3x3_s2"))[:4],
                 p["inception_3a/1x1"][0].reshape(64, 192, 1, 1), p["inception_3a/1x1"][1], 1, 0, relu=True,
                 what="inception_3a/1x1")
    R.check_conv(N(net.blob("inception_4e/output"))[:4, 256:576], N(net.blob("inception_4e/3x3_reduce"))[:4],
                 p["inception_4e/3x3"][0].reshape(320, 160, 3, 3), p["inception_4e/3x3"][1], 1, 1, relu=True,
                 what="inception_4e/3x3")
    mc.close()
    net.close()


def test_c5_conv_fault_extension(rs, oracle_mod):
    """SURVEY.md §7's C5 extension: with fault_layers "InnerProduct,Convolution"
    every Convolution blob is faultable too (the reference faults only the IP
    blobs, net.cpp:484-489).  GoogLeNet b32, per-layer SA ratios (convolution
    weights 30/40/30, IP 20/60/20): every blob of every map bit-exact against
    the oracle's injection with its broken count exact; over 3 maps each conv
    weight blob's broken fraction and -1/0/+1 split inside the 3.8 sigma bound;
    and the forward after injection runs on the injected weights — the first
    fault layer is now conv1, so the MC driver's injection overlap has nothing
    to hide under, and any packed-weight reuse would show up as a stale
    convolution (conv1/7x7_s2 and inception_4a/5x5 within 1e-4 of Σ|a·b| of a
    float64 evaluation with the injected weights)."""
    from rramsim import make_inject_cfg
    caffe, models = rs
    B = 32
    net = caffe.Net(models.googlenet(test_batch=B), "test",
                    models.net_options("googlenet", fault_layers="InnerProduct,Convolution"))
    layers = net.layers()
    types = {i: t for i, (n, t, k) in enumerate(layers)}
    fps = net.failure_params()
    n_conv = sum(1 for n, t, k in layers if t == "Convolution")
    assert n_conv == 59                                 # trunk 3 + 9 inceptions x 6 + 2 aux heads
    assert len(fps) == 2 * (n_conv + 5)
    assert {types[f["layer_id"]] for f in fps} == {"Convolution", "InnerProduct"}
    p = 0.02
    ratios = [(30, 40, 30) if types[f["layer_id"]] == "Convolution" else (20, 60, 20) for f in fps]
    scale = 7.0
    cfgs = [make_inject_cfg(p, *r, stuck_scale=scale) for r in ratios]
    clean = [N(f["data"]) for f in fps]
    mc = caffe.MonteCarlo(net, cfgs, seed=123, max_maps=8)
    maps = 3
    broken = np.zeros(len(fps), np.int64)
    split = np.zeros((len(fps), 3), np.int64)
    for m in range(maps):
        mc.reset()
        mc.run(m, 1)
        st = mc.stats()
        for i, f in enumerate(fps):
            ref, nb = oracle_mod.inject(clean[i], _oracle_cfg(oracle_mod, cfgs[i]), 123, m, i)
            got = N(f["data"])
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (m, i)
            assert st["broken"][i] == nb, (m, i)
            broken[i] += nb
            if i % 2 == 0:
                g = got[~np.isin(clean[i], [-scale, 0.0, scale])]
                split[i] += [(g == -scale).sum(), (g == 0).sum(), (g == scale).sum()]
        # the forward of this map ran on its injected weights
        pl = _params_by_layer(net)
        R.check_conv(N(net.blob("conv1/7x7_s2"))[:4], N(net.blob("data"))[:4],
                     pl["conv1/7x7_s2"][0].reshape(64, 3, 7, 7), pl["conv1/7x7_s2"][1], 2, 3, relu=True,
                     what=f"conv1/7x7_s2 map {m}")
        R.check_conv(N(net.blob("inception_4a/output"))[:4, 400:448], N(net.blob("inception_4a/5x5_reduce"))[:4],
                     pl["inception_4a/5x5"][0].reshape(48, 16, 5, 5), pl["inception_4a/5x5"][1], 1, 2, relu=True,
                     what=f"inception_4a/5x5 map {m}")
    checked = 0
    for i, f in enumerate(fps):
        if types[f["layer_id"]] != "Convolution" or i % 2:
            continue
        assert _binom_ok(int(broken[i]), maps * f["count"], p), (i, broken[i])
        nb_seen = int(split[i].sum())
        if nb_seen >= 200:
            for c in range(3):
                assert _binom_ok(int(split[i][c]), nb_seen, ratios[i][c] / 100), (i, c, split[i])
            checked += 1
    assert checked >= 20
    mc.close()
    net.close()
