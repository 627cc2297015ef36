"""GPU tests of the remapping / genetic strategies, the
strategy kernels, and the .caffemodel / .solverstate / fault-state files
(§8f-2), through include/rram_caffe.h, checked against the oracle's
restatements of strategy.cpp and against round trips."""
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


# ---------------------------------------------------------------- kernels
def test_stuck_zero_counts_and_permutes(device):
    import torch
    from rramsim import ops
    g = torch.Generator().manual_seed(3)
    rows, cols = 37, 301
    e = torch.where(torch.rand(rows, cols, generator=g) < 0.1, -1.0, 5.0)
    e[0, :5] = 0.0                                     # e == 0 is not failed for remapping (e < 0, Q7)
    v = torch.randint(-1, 2, (rows, cols), generator=g).float()
    rc = torch.zeros(rows, dtype=torch.int32, device=device)
    cc = torch.zeros(cols, dtype=torch.int32, device=device)
    ed, vd = e.to(device), v.to(device)
    ops.stuck_zero_counts(ed, vd, rows, cols, rc, cc)
    flag = (e < 0) & (v == 0)
    assert np.array_equal(N(rc), flag.sum(1).numpy())
    assert np.array_equal(N(cc), flag.sum(0).numpy())
    src = torch.randn(rows, cols, device=device)
    to = torch.randperm(rows, generator=g).int().to(device)
    frm = torch.randperm(rows, generator=g).int().to(device)
    dst = torch.zeros_like(src)
    ops.permute_rows(src, dst, cols, to, frm)
    exp = torch.zeros_like(src)
    exp[to.long()] = src[frm.long()]
    assert torch.equal(dst, exp)
    to_c = torch.randperm(cols, generator=g).int().to(device)
    frm_c = torch.randperm(cols, generator=g).int().to(device)
    dst = torch.zeros_like(src)
    ops.permute_cols(src, dst, rows, cols, to_c, frm_c)
    exp = torch.zeros_like(src)
    exp[:, to_c.long()] = src[:, frm_c.long()]
    assert torch.equal(dst, exp)
    flat = src.reshape(-1)
    out = torch.zeros(rows, device=device)
    ops.permute_elems(flat, out, to, frm)
    assert torch.equal(out[to.long()], flat[frm.long()])


# ---------------------------------------------------------------- helpers
def _fc_state(s):
    """(weights data, diff, bias data, diff, fault e, v) of LeNet's ip1 / ip2."""
    fps = s.net.failure_params()
    fs = s.fail_state()
    shapes = [(500, 800), (500,), (10, 500), (10,)]
    W = [N(fps[i]["data"]).reshape(shapes[i]) for i in range(4)]
    D = [N(fps[i]["diff"]).reshape(shapes[i]) for i in range(4)]
    E = [N(fs[i][0]).reshape(shapes[i]) for i in range(4)]
    V = [N(fs[i][1]).reshape(shapes[i]) for i in range(4)]
    return fps, fs, W, D, E, V


def _set_faults(fs, rng, distinct_rows=True):
    """Fault state with distinct per-neuron stuck-at-zero counts on ip1's rows
    (so std::sort has no ties) plus cells that must not count (v != 0, e == 0)."""
    import torch
    e1 = np.full((500, 800), 1e6, np.float32)
    v1 = rng.integers(-1, 2, (500, 800)).astype(np.float32)
    perm = rng.permutation(500)
    for j in range(500):
        cols = rng.choice(800, size=perm[j], replace=False)
        e1[j, cols] = -5.0
        v1[j, cols] = 0.0
    noise = rng.random((500, 800)) < 0.01          # failed but stuck at +-1: not counted
    e1[noise & (v1 != 0)] = -1.0
    free = np.flatnonzero(e1[0] > 0)[:3]
    e1[0, free], v1[0, free] = 0.0, 0.0             # e == 0 stuck at 0: strict "< 0" (Q7) excludes it
    e2 = np.full((10, 500), 1e6, np.float32)
    v2 = np.ones((10, 500), np.float32)             # ip2 cells all stuck at +1 if failed: no column flags
    e2[rng.random((10, 500)) < 0.05] = -1.0
    for i, (e, v) in ((0, (e1, v1)), (2, (e2, v2))):
        fs[i][0].copy_(torch.from_numpy(e.reshape(-1)))
        fs[i][1].copy_(torch.from_numpy(v.reshape(-1)))


def _lenet_solver(rs, extra="", **kw):
    caffe, models = rs
    sp = models.solver(base_lr=0.01, momentum=0.9, weight_decay=0.0005, max_iter=100,
                       failure_mean=1e6, failure_std=1.0, **kw) + extra
    return caffe.Solver(sp, models.lenet(train_batch=16, test_batch=16), models.net_options("lenet"))


# ---------------------------------------------------------------- remapping
@pytest.mark.parametrize("compat", [False, True])
def test_remapping_apply_matches_oracle(rs, oracle_mod, tmp_path, compat):
    import torch
    rng = np.random.default_rng(11)
    prune = rng.permutation(500)
    pf = tmp_path / "prune_order.txt"
    pf.write_text(" ".join(str(x) for x in prune) + "\n")
    extra = (f'failure_strategy {{ type: "remapping" start: 0 period: 1 prune_order_file: "{pf}" '
             f'rram_reference_compat: {"true" if compat else "false"} }}\n')
    s = _lenet_solver(rs, extra)
    fps, fs, *_ = _fc_state(s)
    _set_faults(fs, rng)
    for f in fps:                                    # a non-trivial diff to move along with the data
        f["diff"].copy_(torch.randn_like(f["diff"]))
    _, _, W, D, E, V = _fc_state(s)
    s.apply_strategies()
    _, _, W2, D2, E2, V2 = _fc_state(s)
    eW, eD, eB, eBd, orders = oracle_mod.remap_apply([W[0], W[2]], [D[0], D[2]], [W[1], W[3]], [D[1], D[3]],
                                                     [E[0], E[2]], [V[0], V[2]], [prune], compat=compat)
    assert np.array_equal(W2[0], eW[0]) and np.array_equal(W2[2], eW[1])
    assert np.array_equal(D2[0], eD[0]) and np.array_equal(D2[2], eD[1])
    assert np.array_equal(W2[1], eB[0]) and np.array_equal(D2[1], eBd[0])
    assert np.array_equal(W2[3], W[3])               # the last layer's bias is never moved
    for a, b in zip(E + V, E2 + V2):                 # physical cells stay where they are
        assert np.array_equal(a, b)
    s.close()


def test_remapping_period_and_start(rs, tmp_path):
    import torch
    pf = tmp_path / "p.txt"
    pf.write_text(" ".join(str(x) for x in range(499, -1, -1)))
    s = _lenet_solver(rs, f'failure_strategy {{ type: "remapping" start: 2 period: 3 prune_order_file: "{pf}" }}\n')
    fps = s.net.failure_params()
    applied = []
    for t in range(1, 9):
        w0 = N(fps[0]["data"])
        s.apply_strategies()
        applied.append(not np.array_equal(w0, N(fps[0]["data"])))
    # times_ in 1..8: applied when times_ >= start and (times_ - start) % period == 0 -> 2, 5, 8
    assert applied == [False, True, False, False, True, False, False, True]
    s.close()


def test_remapping_bad_prune_file_fails_cleanly(rs, tmp_path):
    caffe, _ = rs
    from rramsim._kernels import RramError
    pf = tmp_path / "short.txt"
    pf.write_text("1 2 3")
    with pytest.raises(RramError, match="prune order file not correct"):
        _lenet_solver(rs, f'failure_strategy {{ type: "remapping" prune_order_file: "{pf}" }}\n')
    with pytest.raises(RramError, match="No strategy named"):
        _lenet_solver(rs, 'failure_strategy { type: "bogus" }\n')


# ---------------------------------------------------------------- genetic
@pytest.mark.parametrize("compat", [False, True])
def test_genetic_apply_matches_oracle(rs, oracle_mod, tmp_path, compat):
    import torch
    caffe, models = rs
    rng = np.random.default_rng(5)
    # prune net: LeNet TEST with about half of the IP weights pruned (exact zeros)
    net_txt = tmp_path / "prune_net.prototxt"
    net_txt.write_text(models.lenet(train_batch=16, test_batch=16))
    pnet = caffe.Net(models.lenet(train_batch=16, test_batch=16), "test", models.net_options("lenet"))
    for f in pnet.failure_params():
        d = f["data"]
        d.mul_((torch.rand_like(d) < 0.5).float())
    model = tmp_path / "prune.caffemodel"
    pnet.save(model)
    prune = [N(f["data"]) for f in pnet.failure_params()]
    pnet.close()
    extra = (f'failure_strategy {{ type: "genetic" start: 0 period: 1 switch_time: 300 '
             f'prune_net_file: "{net_txt}" prune_model_file: "{model}" '
             f'rram_reference_compat: {"true" if compat else "false"} }}\n')
    s = _lenet_solver(rs, extra)
    fps = s.net.failure_params()
    fs = s.fail_state()
    for i, (e, v) in enumerate(fs):
        ee = np.where(rng.random(e.numel()) < 0.2, -3.0, 1e6).astype(np.float32)
        e.copy_(torch.from_numpy(ee))
    for f in fps:
        f["diff"].copy_(torch.randn_like(f["diff"]))
    shapes = [(500, 800), (500,), (10, 500), (10,)]
    weights = [(N(f["data"]), N(f["diff"]), shapes[i]) for i, f in enumerate(fps)]
    fail_e = [N(e) for e, _ in fs]
    r = iter(caffe.glibc_rand(1, 100000))
    Wt, P, before, after, accepted = oracle_mod.genetic_apply([0, 2], fail_e, prune, weights, lambda: next(r),
                                                              300, compat=compat)
    s.apply_strategies()
    typ, b, a, acc = s.strategy_info(0)
    assert typ == "genetic"
    assert (b, a, acc) == (before, after, accepted)
    assert accepted > 0 and after < before
    for i, f in enumerate(fps):
        assert np.array_equal(N(f["data"]), Wt[i][0]), i
        assert np.array_equal(N(f["diff"]), Wt[i][1]), i
    assert any("dist: before:" in l for l in s.log_lines)
    s.close()


# ------------------------------------------------------------ weight files
def test_caffemodel_save_load_round_trip(rs, tmp_path):
    import torch
    caffe, models = rs
    a = caffe.Net(models.lenet(test_batch=4), "test", models.net_options("lenet"))
    for p in a.params():
        p["data"].copy_(torch.randn_like(p["data"]))
    f = tmp_path / "w.caffemodel"
    a.save(f)
    desc = caffe.caffemodel_describe(f)
    assert [d[0] for d in desc if d[2] == 0] == ["conv1", "conv2", "ip1", "ip2"]
    caffe.set_random_seed(99)
    b = caffe.Net(models.lenet(test_batch=4), "test", models.net_options("lenet"))
    assert not all(torch.equal(x["data"], y["data"]) for x, y in zip(a.params(), b.params()))
    b.copy_from(f)
    for x, y in zip(a.params(), b.params()):
        assert torch.equal(x["data"], y["data"])
    b.blob("data").copy_(a.blob("data"))             # synthetic data differs with the seed
    a.forward()
    b.forward()
    assert torch.equal(a.blob("ip2"), b.blob("ip2"))
    # shape mismatch is a clean error, not an abort
    from rramsim._kernels import RramError
    c = caffe.Net(models.cifar10_quick(test_batch=2), "test", models.net_options("cifar10_quick"))
    bad = tmp_path / "bad.caffemodel"
    c.save(bad)                                      # same layer names (conv1, ip1, ...), other shapes
    with pytest.raises(RramError, match="shape mismatch|Incompatible"):
        b.copy_from(bad)
    for n in (a, b, c):
        n.close()
    caffe.set_random_seed(1701)


def test_golden_caffemodel_loads_into_net(rs, tmp_path):
    """The protobuf-serialised fixture loads by layer name (V2 and V1 files)."""
    caffe, _ = rs
    from pathlib import Path
    gold = Path(__file__).resolve().parent / "golden"
    net_txt = """name: "tiny"
layer { name: "data" type: "Input" top: "data" input_param { shape { dim: 2 dim: 4 } } }
layer { name: "ip1" type: "InnerProduct" bottom: "data" top: "ip1" inner_product_param { num_output: 3 } }
layer { name: "relu1" type: "ReLU" bottom: "ip1" top: "ip1" }
layer { name: "ip2" type: "InnerProduct" bottom: "ip1" top: "ip2" inner_product_param { num_output: 2 } }
"""
    net = caffe.Net(net_txt, "test")
    net.copy_from(gold / "tiny_net.caffemodel")

    def vals(n, seed):
        return np.array([((i * 37 + seed * 11) % 257 - 128) / 64.0 for i in range(n)], np.float32)
    ps = net.params()
    exp = [vals(12, 0), vals(3, 1), vals(6, 20), vals(2, 21)]
    for p, e in zip(ps, exp):
        assert np.array_equal(N(p["data"]), e)
    assert np.array_equal(N(ps[2]["diff"]), vals(6, 99))
    net.close()


# ----------------------------------------------------- snapshot / restore
@pytest.mark.parametrize("fmt", ["BINARYPROTO", "HDF5"])
def test_snapshot_restore_resumes_bit_exact(rs, tmp_path, fmt):
    """Snapshot at iter 3 (weights, momentum history, fault maps), restore into
    a fresh solver, continue: identical to the uninterrupted run, in both of
    the reference's snapshot formats (solver.cpp:461-530, sgd_solver.cpp:249-351;
    cifar10_full_solver.prototxt itself asks for HDF5)."""
    caffe, models = rs
    prefix = tmp_path / "snap"
    extra = f'snapshot_prefix: "{prefix}"\nsnapshot_format: {fmt}\n'
    h5 = ".h5" if fmt == "HDF5" else ""
    kw = dict(failure_mean=300.0, failure_std=200.0, failure_prob=(10, 20, 10))

    def make(seed):
        caffe.set_random_seed(seed)
        sp = models.solver(base_lr=0.01, momentum=0.9, weight_decay=0.0005, max_iter=100, **kw) + extra
        return caffe.Solver(sp, models.lenet(train_batch=16, test_batch=16), models.net_options("lenet"))
    a = make(5)
    a.step(3)
    state = a.snapshot()
    assert state.endswith("snap_iter_3.solverstate" + h5)
    for ext in (".caffemodel" + h5, ".solverstate" + h5, ".faultstate"):
        assert (tmp_path / f"snap_iter_3{ext}").exists()
    a.step(2)
    b = make(5)                                      # same synthetic data; scramble what restore must bring back
    import torch
    for p in b.net.params():
        p["data"].copy_(torch.randn_like(p["data"]))
    for e, v in b.fail_state():
        e.copy_(torch.rand_like(e) * 1e3)
        v.zero_()
    b.restore(state)
    assert b.iter == 3
    b.step(2)
    for x, y in zip(a.net.params(), b.net.params()):
        assert np.array_equal(N(x["data"]), N(y["data"]))
    for (ea, va), (eb, vb) in zip(a.fail_state(), b.fail_state()):
        assert np.array_equal(N(ea), N(eb)) and np.array_equal(N(va), N(vb))
    assert any("Snapshotting solver state" in l for l in a.log_lines)
    a.close()
    b.close()
    caffe.set_random_seed(1701)
