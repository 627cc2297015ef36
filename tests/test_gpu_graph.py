"""hipGraph replay of Monte-Carlo maps (include/rram_caffe.h rram_mc_set_graph;
no reference counterpart: the reference runs one map per process,
SURVEY.md §3.3).  One map (injection + forward + statistics) is captured
after one eager map and replayed, the map id and the per-map row advancing
in device memory.  Gate: bit-identity with the eager maps — per-map
accuracy / loss, broken-cell counts, the last map's weights and logits —
over consecutive and strided map ids (the bench's map m on rank m mod N),
and with the conv-fault extension, whose injections rewrite the conv
weights every map (the captured map repacks them)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def N(t):
    import torch
    torch.cuda.synchronize()
    return t.detach().cpu().numpy().copy()


def _run(model, graph, calls, opts_extra=None, cfg_kw=None, release=False):
    import torch
    from rramsim import caffe, kernels, make_inject_cfg, models
    caffe.set_stream_from_torch()
    caffe.set_random_seed(1701)
    name = "cifar10_quick" if model == "cifar" else "lenet"
    build = models.cifar10_quick if model == "cifar" else models.lenet
    opts = models.net_options(name, **(opts_extra or {}))
    net = caffe.Net(build(test_batch=50), "test", opts)
    mc = caffe.MonteCarlo(net, make_inject_cfg(0.05, **(cfg_kw or {})), seed=77, max_maps=64)
    mc.set_graph(graph)
    for begin, count in calls:
        mc.run(begin, count)
        if release:                        # gather tables freed between runs
            torch.cuda.synchronize()
            kernels.check(kernels.load().rram_release_caches(), "release_caches")
    st = mc.stats()
    fps = [N(f["data"]) for f in net.failure_params()]
    outs = {k: N(v) for k, v in net.outputs().items()}
    active = mc.graph_active()
    mc.close()
    net.close()
    return st, fps, outs, active


@pytest.mark.parametrize("model", ["lenet", "cifar"])
@pytest.mark.parametrize("calls", [[(0, 6)], [(0, 1), (2, 1), (4, 1), (6, 1)], [(3, 2), (10, 3)]],
                         ids=["consecutive", "strided", "two_runs"])
def test_graph_maps_equal_eager(device, model, calls):
    ref = _run(model, False, calls)
    got = _run(model, True, calls)
    assert got[3] and not ref[3]                      # the graph ran
    assert got[0]["per_map"] == ref[0]["per_map"]
    assert got[0]["broken"] == ref[0]["broken"] and got[0]["sums"] == ref[0]["sums"]
    assert got[0]["maps"] == ref[0]["maps"]
    for a, b in zip(got[1], ref[1]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    for k in ref[2]:
        assert np.array_equal(got[2][k], ref[2][k]), k


def test_graph_maps_release_caches_between_runs(device):
    """rram_release_caches between MonteCarlo::Run calls: after
    the eager warm-up map (a one-map run) and after a captured graph, the
    moved scratch generation sends the next map down the eager path (the
    freed gather tables are rebuilt outside any capture) and the one after
    recaptures; per-map statistics and weights equal the eager maps."""
    calls = [(0, 1), (1, 1), (2, 3), (5, 2)]
    ref = _run("cifar", False, calls, release=True)
    got = _run("cifar", True, calls, release=True)
    assert got[3]
    assert got[0]["per_map"] == ref[0]["per_map"] and got[0]["broken"] == ref[0]["broken"]
    for a, b in zip(got[1], ref[1]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_graph_conv_fault_extension_equals_eager(device):
    calls = [(0, 4)]
    kw = dict(opts_extra=dict(fault_layers="InnerProduct,Convolution"))
    ref = _run("cifar", False, calls, **kw)
    got = _run("cifar", True, calls, **kw)
    assert got[3]
    assert got[0]["per_map"] == ref[0]["per_map"] and got[0]["broken"] == ref[0]["broken"]
    for k in ref[2]:
        assert np.array_equal(got[2][k], ref[2][k]), k


def test_graph_quantised_lognormal_equals_eager(device):
    """C2's injection modes (quantisation + lognormal variation)."""
    calls = [(0, 5)]
    kw = dict(cfg_kw=dict(quant_levels=16, g_max=0.5, var_sigma=0.1))
    ref = _run("cifar", False, calls, **kw)
    got = _run("cifar", True, calls, **kw)
    assert got[3]
    assert got[0]["per_map"] == ref[0]["per_map"] and got[0]["broken"] == ref[0]["broken"]
    for a, b in zip(got[1], ref[1]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _train(graph, iters, lr_policy="fixed", test_batch=20, side_stream=False, release=False, **kw):
    import contextlib
    import torch
    from rramsim import caffe, models, kernels
    ctx = torch.cuda.stream(torch.cuda.Stream()) if side_stream else contextlib.nullcontext()
    with ctx:
        caffe.set_stream_from_torch()
        caffe.set_random_seed(1701)
        sp = models.solver(base_lr=0.001, momentum=0.9, weight_decay=0.004, lr_policy=lr_policy, max_iter=1000,
                           failure_mean=5e4, failure_std=1.5e4, failure_prob=(5, 90, 5), threshold=0.001, **kw)
        s = caffe.Solver(sp, models.cifar10_full(train_batch=20, test_batch=test_batch),
                         dict(models.net_options("cifar10_full"), fused_update=True))
        s.set_graph(graph)
        for n in iters:
            s.step(n)
            if release:                                 # gather tables freed between replays
                torch.cuda.synchronize()
                kernels.check(kernels.load().rram_release_caches(), "release_caches")
        ps = [N(p["data"]) for p in s.net.params()]
        hist = [N(h) for h in s.history()]
        fs = s.fail_state()
        st = (ps, hist, [N(e) for e, v in fs], s.broken_counts(), s.graph_active())
        s.close()
    caffe.set_stream_from_torch()
    return st


@pytest.mark.parametrize("policy", [dict(), dict(lr_policy="step", gamma=0.5, stepsize=4)], ids=["fixed", "step"])
def test_graph_training_equals_eager(device, policy):
    """C4's fault-aware training (fused update + threshold + Fail): 10
    iterations in three step() calls replayed as graphs equal the eager
    iterations bit for bit — weights, momentum history, endurance, broken
    counts; the step policy's rate change at iteration 4 / 8 recaptures."""
    ref = _train(False, [3, 4, 3], **policy)
    got = _train(True, [3, 4, 3], **policy)
    assert got[4] and not ref[4]
    for a, b in zip(got[0] + got[1] + got[2], ref[0] + ref[1] + ref[2]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert got[3] == ref[3]


@pytest.mark.parametrize("mode", ["test_interval", "display", "average_loss", "side_stream", "release_caches"])
def test_graph_training_interleaved_equals_eager(device, mode):
    """Graph iterations interleaved with the eager work that breaks a replay
    (ADVICE r04): TestAll every 3 iterations on a larger test batch (its
    forward grows the shared workspace / pack buffers the captured launches
    point into: the scratch generation in Solver::graph_key recaptures),
    display iterations (eager), average_loss > 1 (no graph at all), and a
    non-NULL caller stream (captured directly on it), and the gather tables
    freed between step() calls (rram_release_caches, ADVICE r05: the changed
    key drops the graphs and that iteration runs eager, rebuilding the tables
    outside any capture; the next one recaptures).  Every variant equals
    the eager run bit for bit."""
    kw = dict(test_interval=dict(test_interval=3, test_iter=1, test_batch=100),
              display=dict(display=2),
              average_loss=dict(display=2, average_loss=2),
              side_stream=dict(side_stream=True),
              release_caches=dict(release=True))[mode]
    iters = [4, 5] if mode != "release_caches" else [3, 1, 1, 3, 2]
    ref = _train(False, iters, **kw)
    got = _train(True, iters, **kw)
    if mode != "average_loss":
        assert got[4]                                   # the graph ran
    for a, b in zip(got[0] + got[1] + got[2], ref[0] + ref[1] + ref[2]):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert got[3] == ref[3]


def test_graph_maps_with_pooled_output_fold_read_between_runs(device):
    """AlexNet (LRN + max pool folds, the pooled-output fold on): maps
    replayed from a graph, pool1 read through the C-ABI between two runs
    (materialised; the fold is undone, which must force a recapture: the
    captured map skips the fp32 pooled top), then more maps: per-map
    statistics, broken counts, pool1 and the outputs bit-identical to the
    eager sequence."""
    import torch
    from rramsim import caffe, make_inject_cfg, models

    def run(graph):
        caffe.set_stream_from_torch()
        caffe.set_random_seed(1701)
        net = caffe.Net(models.alexnet(test_batch=4), "test", models.net_options("alexnet"))
        mc = caffe.MonteCarlo(net, make_inject_cfg(0.05), seed=77, max_maps=16)
        mc.set_graph(graph)
        mc.run(0, 3)
        torch.cuda.synchronize()
        p1 = N(net.blob("pool1"))
        mc.run(3, 3)
        torch.cuda.synchronize()
        p2 = N(net.blob("pool1"))
        st = mc.stats()
        outs = {k: N(v) for k, v in net.outputs().items()}
        active = mc.graph_active()
        mc.close()
        net.close()
        return st, p1, p2, outs, active

    ref = run(False)
    got = run(True)
    assert got[4] and not ref[4]
    assert got[0]["per_map"] == ref[0]["per_map"] and got[0]["broken"] == ref[0]["broken"]
    assert np.array_equal(got[1], ref[1]) and np.array_equal(got[2], ref[2])
    for k in ref[3]:
        assert np.array_equal(got[3][k], ref[3][k]), k
