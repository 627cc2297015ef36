"""GPU tests of the C++ host runtime (Net / Solver / FailureMaker / MonteCarlo)
through include/rram_caffe.h, checked against the CPU oracle."""
import math

import numpy as np
import pytest

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


def test_lenet_forward_matches_oracle(rs, oracle_mod):
    caffe, models = rs
    net = caffe.Net(models.lenet(test_batch=16), "test", models.net_options("lenet"))
    net.forward()
    p = _params_by_layer(net)
    x = N(net.blob("data")).reshape(16, 1, 28, 28)
    label = N(net.blob("label")).reshape(16)
    assert x.min() >= 0 and x.max() < 1.0 and np.allclose(x * 256, np.round(x * 256))
    y = oracle_mod.conv_im2col(x, p["conv1"][0].reshape(20, 1, 5, 5), p["conv1"][1])
    y = oracle_mod.pool(y, 2, 2)
    y = oracle_mod.conv_im2col(y, p["conv2"][0].reshape(50, 20, 5, 5), p["conv2"][1])
    y = oracle_mod.pool(y, 2, 2).reshape(16, -1)
    y = np.maximum(y @ p["ip1"][0].reshape(500, 800).T + p["ip1"][1], 0)
    y = y @ p["ip2"][0].reshape(10, 500).T + p["ip2"][1]
    got = N(net.blob("ip2")).reshape(16, 10)
    np.testing.assert_allclose(got, y, rtol=1e-4, atol=1e-4)
    out = {k: float(N(v)[0]) for k, v in net.outputs().items()}
    assert out["accuracy"] == oracle_mod.accuracy(got, label) / 16
    assert abs(out["loss"] - oracle_mod.softmax_loss(oracle_mod.softmax(got), label)) < 1e-4
    net.close()


def test_alexnet_forward_matches_oracle(rs, oracle_mod):
    caffe, models = rs
    B = 2
    net = caffe.Net(models.alexnet(test_batch=B), "test", models.net_options("alexnet"))
    net.forward()
    p = _params_by_layer(net)
    x = N(net.blob("data")).reshape(B, 3, 227, 227)
    sh = {"conv1": (96, 3, 11, 11), "conv2": (256, 48, 5, 5), "conv3": (384, 256, 3, 3),
          "conv4": (384, 192, 3, 3), "conv5": (256, 192, 3, 3)}
    cw = {k: p[k][0].reshape(v) for k, v in sh.items()}
    y = oracle_mod.relu(oracle_mod.conv_im2col(x, cw["conv1"], p["conv1"][1], 4, 0))
    y = oracle_mod.pool(oracle_mod.lrn(y, 5, 1e-4, 0.75), 3, 2)
    y = oracle_mod.relu(oracle_mod.conv_im2col(y, cw["conv2"], p["conv2"][1], 1, 2, 1, 2))
    y = oracle_mod.pool(oracle_mod.lrn(y, 5, 1e-4, 0.75), 3, 2)
    y = oracle_mod.relu(oracle_mod.conv_im2col(y, cw["conv3"], p["conv3"][1], 1, 1))
    y = oracle_mod.relu(oracle_mod.conv_im2col(y, cw["conv4"], p["conv4"][1], 1, 1, 1, 2))
    y = oracle_mod.relu(oracle_mod.conv_im2col(y, cw["conv5"], p["conv5"][1], 1, 1, 1, 2))
    np.testing.assert_allclose(N(net.blob("conv5")).reshape(y.shape), y, rtol=1e-3, atol=1e-3)
    y = oracle_mod.pool(y, 3, 2).reshape(B, -1)
    for k, n in (("fc6", 4096), ("fc7", 4096), ("fc8", 1000)):
        y = y @ p[k][0].reshape(n, -1).T + p[k][1]
        if k != "fc8":
            y = np.maximum(y, 0)
    got = N(net.blob("fc8")).reshape(B, 1000)
    np.testing.assert_allclose(got, y, rtol=1e-3, atol=1e-3)
    names = [n for n, _, _ in net.layers()]
    assert len(net.failure_params()) == 6          # fc6/fc7/fc8 weights + biases (net.cpp:484-489)
    assert sum(f["count"] for f in net.failure_params()) == 58_631_144
    assert "conv1" in names
    net.close()


@pytest.mark.parametrize("name", ["cifar10_quick", "cifar10_full", "caffenet", "googlenet"])
def test_config_nets_build_and_forward(rs, name):
    caffe, models = rs
    f, _, _ = models.CONFIGS[name]
    net = caffe.Net(f(test_batch=4), "test", models.net_options(name))
    loss = net.forward()
    assert np.isfinite(loss)
    outs = {k: float(N(v)[0]) for k, v in net.outputs().items()}
    for k, v in outs.items():
        assert np.isfinite(v), k
    net.close()


def _lenet_solver(rs, **kw):
    caffe, models = rs
    sp = models.solver(base_lr=0.01, momentum=0.9, weight_decay=0.0005, lr_policy="inv", gamma=0.0001,
                       power=0.75, max_iter=100, **kw)
    return caffe.Solver(sp, models.lenet(train_batch=32, test_batch=32), models.net_options("lenet"))


def test_solver_fail_step_bit_exact(rs, oracle_mod):
    """One Solver::Step in the fork's order (solver.cpp:300-305): after the
    step, fault state and IP weights equal the oracle's Fail_cpu applied to
    (w - update, endurance_before, values) with the update left in diff."""
    s = _lenet_solver(rs, failure_mean=150.0, failure_std=100.0, failure_prob=(10, 20, 10))
    net = s.net
    fps = net.failure_params()
    fs = s.fail_state()
    assert len(fps) == len(fs) == 4
    e0 = [N(e) for e, _ in fs]
    v0 = [N(v) for _, v in fs]
    w0 = [N(f["data"]) for f in fps]
    s.step(1)
    for i, f in enumerate(fps):
        dw = N(f["diff"])
        w_exp, e_exp, nb = oracle_mod.fail_apply(dw, (w0[i] - dw).astype(np.float32), e0[i], v0[i])
        assert np.array_equal(N(f["data"]).view(np.uint32), w_exp.view(np.uint32)), i
        assert np.array_equal(N(fs[i][0]).view(np.uint32), e_exp.view(np.uint32)), i
        assert s.broken_counts()[i] == nb
    # the initial broken fraction follows P(e <= 0) = Phi(-mean/std)
    from rramsim import gaussian_fault_rate
    n = sum(len(e) for e in e0)
    p = gaussian_fault_rate(150.0, 100.0)
    frac = sum(int((e <= 0).sum()) for e in e0) / n
    assert abs(frac - p) <= 3.8 * math.sqrt(p * (1 - p) / n)
    s.close()


def test_threshold_strategy_in_solver(rs, oracle_mod):
    s = _lenet_solver(rs, failure_mean=1e9, failure_std=1.0, threshold=1e9)   # nothing breaks, all IP updates cleared
    fps = s.net.failure_params()
    w0 = [N(f["data"]) for f in fps]
    s.step(2)
    for i, f in enumerate(fps):
        assert np.array_equal(N(f["data"]), w0[i])
        assert not N(f["diff"]).any()
    # conv params still train
    ps = s.net.params()
    assert N(ps[0]["diff"]).any()
    s.close()


def _run_solver_state(caffe, models, fused, steps, extra="", net="lenet", seed=77, **kw):
    caffe.set_random_seed(seed)
    sp = models.solver(base_lr=0.01, momentum=0.9, weight_decay=0.0005, max_iter=10, **kw) + extra
    f, _, _ = models.CONFIGS[net]
    s = caffe.Solver(sp, f(train_batch=32, test_batch=32), models.net_options(net, fused_update=fused))
    s.step(steps)
    out = ([N(p["data"]) for p in s.net.params()], [N(e) for e, _ in s.fail_state()], s.broken_counts())
    s.close()
    return out


def _assert_states_bit_equal(a, b):
    for x, y in zip(a[0], b[0]):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
    for x, y in zip(a[1], b[1]):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
    assert a[2] == b[2]


def test_fused_tail_matches_reference_order(rs):
    """The fused Regularize + SGDUpdate + threshold + Update + Fail pass gives
    the same bits as the reference order ComputeUpdate -> ApplyStrategy ->
    ApplyUpdate -> Fail (solver.cpp:300-305): weights, endurance, counts."""
    caffe, models = rs
    kw = dict(failure_mean=300.0, failure_std=200.0, threshold=0.001)
    ref = _run_solver_state(caffe, models, False, 4, **kw)
    fused = _run_solver_state(caffe, models, True, 4, **kw)
    _assert_states_bit_equal(ref, fused)
    assert sum(ref[2]) > 0                              # some cells broke along the way


def test_flip_cache_same_bits(rs):
    """The fused update writes each stride-1 convolution's flipped kernel next
    to its weights (rram_update_seg.w_flip) and the next backward of the same
    Step call reads it instead of flipping (conv_layer.cu:47-52's data
    gradient as a forward convolution): CIFAR-10 full (conv2 / conv3 take it),
    two Step calls (the second starts on the flip pass again), bit-identical
    weights, endurance and counts with the cache off."""
    caffe, models = rs

    def run(cache):
        caffe.set_random_seed(31)
        sp = models.solver(base_lr=0.001, momentum=0.9, weight_decay=0.004, max_iter=100,
                           failure_mean=2e3, failure_std=1e3, failure_prob=(5, 90, 5), threshold=0.001)
        f, _, _ = models.CONFIGS["cifar10_full"]
        s = caffe.Solver(sp, f(train_batch=32, test_batch=32),
                         models.net_options("cifar10_full", fused_update=True, conv_flip_cache=cache))
        s.step(3)
        s.step(2)
        out = ([N(p["data"]) for p in s.net.params()], [N(e) for e, _ in s.fail_state()], s.broken_counts())
        s.close()
        return out

    on, off = run(True), run(False)
    _assert_states_bit_equal(on, off)
    assert sum(on[2]) > 0


def test_fused_flag_with_remapping_runs_reference_order(rs, tmp_path):
    """[threshold, remapping] cannot be fused: fused_update=true must fall back
    to the reference order and give exactly the unfused result."""
    caffe, models = rs
    pf = tmp_path / "prune_order.txt"
    pf.write_text(" ".join(str(x) for x in np.random.default_rng(3).permutation(500)) + "\n")
    extra = f'failure_strategy {{ type: "remapping" start: 0 period: 1 prune_order_file: "{pf}" }}\n'
    kw = dict(failure_mean=300.0, failure_std=200.0, threshold=0.001)
    ref = _run_solver_state(caffe, models, False, 3, extra, **kw)
    fused = _run_solver_state(caffe, models, True, 3, extra, **kw)
    _assert_states_bit_equal(ref, fused)


def test_solver_trains_and_tests(rs):
    s = _lenet_solver(rs, test_iter=2, display=5)
    s.step(20)
    assert s.iter == 20
    scores = s.test(0)
    assert len(scores) == 2 and 0.0 <= scores[0] <= 1.0 and np.isfinite(scores[1])
    assert any(l.startswith("Iteration 5, loss = ") for l in s.log_lines)
    assert any("Test net output #0: accuracy = " in l for l in s.log_lines)
    s.close()


def test_mc_matches_manual_inject_and_forward(rs):
    import torch
    caffe, models = rs
    from rramsim import make_inject_cfg, ops
    net = caffe.Net(models.lenet(test_batch=64), "test", models.net_options("lenet"))
    clean = [f["data"].clone() for f in net.failure_params()]
    net.forward()
    clean_out = {k: float(N(v)[0]) for k, v in net.outputs().items()}
    cfg = make_inject_cfg(0.05, 5, 90, 5)
    mc = caffe.MonteCarlo(net, cfg, seed=99, max_maps=16)
    mc.run(0, 4)
    st = mc.stats()
    assert st["maps"] == 4 and len(st["per_map"]) == 4
    # map 2 by hand: inject with the kernel C-ABI + forward
    mc.restore_clean()
    fps = net.failure_params()
    for i, f in enumerate(fps):
        ops.inject(clean[i], f["data"], cfg, 99, 2, i)
    net.forward()
    manual = [float(N(v)[0]) for v in net.outputs().values()]
    np.testing.assert_allclose(manual, st["per_map"][2], rtol=1e-6, atol=1e-6)
    # p = 0 reproduces the clean net exactly
    mc.close()
    for f, c in zip(net.failure_params(), clean):
        assert torch.equal(f["data"], c)               # destroy restores clean weights
    mc0 = caffe.MonteCarlo(net, make_inject_cfg(0.0), seed=1, max_maps=4)
    mc0.run(0, 2)
    st0 = mc0.stats()
    assert st0["broken"] == [0] * len(fps)
    assert st0["per_map"][0] == st0["per_map"][1] == [clean_out[k] for k in net.outputs().keys()]
    mc0.close()
    net.close()


def test_mc_broken_fraction_binomial(rs):
    caffe, models = rs
    from rramsim import make_inject_cfg
    net = caffe.Net(models.lenet(test_batch=8), "test", models.net_options("lenet"))
    n = sum(f["count"] for f in net.failure_params())
    p = 0.02
    mc = caffe.MonteCarlo(net, make_inject_cfg(p), seed=5, max_maps=64)
    mc.run(0, 50)
    st = mc.stats()
    tot = 50 * n
    assert abs(sum(st["broken"]) / tot - p) <= 3.8 * math.sqrt(p * (1 - p) / tot)
    # per-map statistics and the reference's Test-net log lines (plot_pic.py's regex)
    sm = mc.summary()
    acc = [row[0] for row in st["per_map"]]
    assert sm["accuracy"]["maps"] == 50
    assert abs(sm["accuracy"]["mean"] - sum(acc) / 50) < 1e-6
    assert abs(sm["accuracy"]["std"] - float(np.std(acc, ddof=1))) < 1e-5
    assert abs(sm["accuracy"]["ci"] - 1.96 * float(np.std(acc, ddof=1)) / math.sqrt(50)) < 1e-5
    import re
    text = "\n".join(mc.log_lines(100))
    m = re.search(r"accuracy = (?P<acc>[\d\.]+).*?loss = (?P<loss>[\d\.]+)", text, re.DOTALL)
    assert m and abs(float(m.group("acc")) - sm["accuracy"]["mean"]) < 1e-4
    mc.close()
    net.close()


def test_layer_timing_and_flat_params(rs):
    import torch
    caffe, models = rs
    net = caffe.Net(models.lenet(train_batch=16), "train", models.net_options("lenet"))
    net.set_timing(True)
    net.forward()
    net.forward()
    lt = net.layer_times(reset=True)
    assert all(c == 2 for _, _, _, c in lt) and sum(ms for _, _, ms, _ in lt) > 0
    net.set_timing_layer("conv2")                      # one layer's events only (bench.py's timed region)
    net.forward()
    lt = net.layer_times(reset=True)
    assert [(n, c) for n, _, ms, c in lt if c] == [("conv2", 1)] and [ms for n, _, ms, _ in lt if n == "conv2"][0] > 0
    with pytest.raises(KeyError):
        net.set_timing_layer("no_such_layer")
    net.set_timing(False)
    n = net.flat_param_count()
    data = torch.empty(n, device="cuda")
    diff = torch.empty(n, device="cuda")
    before = torch.cat([p["data"].clone() for p in net.params()])
    net.alias_flat_params(data, diff)
    assert torch.equal(data, before)
    net.clear_param_diffs()
    net.forward()
    net.backward()
    torch.cuda.synchronize()
    assert float(diff.abs().sum()) > 0                 # gradients land in the flat buffer
    net.close()
