"""The reference's own solver known-answer tests, on the reference's own data.

src/caffe/test/test_gradient_based_solver.cpp trains a one-output
InnerProduct + EuclideanLoss net on tests/golden/solver_data.h5 (a copy of
src/caffe/test/test_data/solver_data.h5: data 8x3x10x10, targets 8x1, read
through the HDF5Data layer, batch 4) and checks every SGD step against the
analytic least-squares update computed from the net's own state:

    E = 1/(2n) ||X w - y||^2 + lambda/2 ||w||^2
    grad = 1/n (X^T X w - X^T y) + lambda w,  update = lr*grad + mom*history

(ComputeLeastSquaresUpdate / CheckLeastSquaresUpdate, :224-397; tolerance
max(1e-7, 1e-2 * min(|expected|, |solver|)), the reference's).  The SGD cases
of :574-695 are restated below one for one: plain, LR 1/100, weight decay,
momentum, multi-iteration, "everything", weight sharing (Slice + two
InnerProducts sharing `weights` / `bias` + Concat), iter_size accumulation
(CheckAccumulation, :399-436) and snapshot -> restore -> continue (TestSnapshot,
:490-558, EXPECT_EQ: bit for bit).  The multi-device pass of
TestLeastSquaresUpdate (:456-486, P2PSync over 2 GPUs) runs as the
data-parallel solver with 2 ranks on this box's GPU (gloo carries the
collective here) and, with RCCL, as a world-size-1 `nccl` process group.

This pins row a4 (SGD update + Blob::Update), a7 (InnerProduct forward /
backward) and a10 (the data-parallel gradient average) against data and
arithmetic the reference itself ships.  The analytic update is evaluated in
float64 (the reference evaluates the same formula in Dtype loops; the 1e-2
tolerance covers either).
"""
import os
import socket
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
H5 = ROOT / "tests" / "golden" / "solver_data.h5"
NUM, D = 4, 3 * 10 * 10
K_PRECISION, K_MIN_PRECISION = 1e-2, 1e-7     # test_gradient_based_solver.cpp:363-364


def _list_file(tmp_path):
    p = Path(tmp_path) / "solver_data_list.txt"
    p.write_text(f"{H5}\n")
    return str(p)


def net_proto(list_file, batch, share=False):
    """RunLeastSquaresSolver's net_param (test_gradient_based_solver.cpp:87-172)."""
    ip = ('layer {{ name: "{name}" type: "InnerProduct" param {{ name: "weights" }} param {{ name: "bias" }} '
          'inner_product_param {{ num_output: 1 weight_filler {{ type: "gaussian" std: 1.0 }} '
          'bias_filler {{ type: "gaussian" std: 1.0 }} }} bottom: "{bottom}" top: "{top}" }}\n')
    s = ('name: "TestNetwork"\n'
         f'layer {{ name: "data" type: "HDF5Data" hdf5_data_param {{ source: "{list_file}" batch_size: {batch} }} '
         'top: "data" top: "targets" }\n')
    if share:
        s += 'layer { name: "slice" type: "Slice" bottom: "data" top: "data1" top: "data2" slice_param { axis: 0 } }\n'
        s += ip.format(name="innerprod", bottom="data1", top="innerprod1")
        s += ip.format(name="innerprod2", bottom="data2", top="innerprod2")
        s += ('layer { name: "concat" type: "Concat" bottom: "innerprod1" bottom: "innerprod2" top: "innerprod" '
              'concat_param { axis: 0 } }\n')
    else:
        s += ip.format(name="innerprod", bottom="data", top="innerprod")
    s += 'layer { name: "loss" type: "EuclideanLoss" bottom: "innerprod" bottom: "targets" }\n'
    return s


def solver_proto(lr, wd, mom, max_iter, iter_size=1, snapshot=0, prefix=None):
    s = f'max_iter: {max_iter} base_lr: {lr} lr_policy: "fixed" iter_size: {iter_size} random_seed: 1701\n'
    if wd != 0:
        s += f"weight_decay: {wd}\n"
    if mom != 0:
        s += f"momentum: {mom}\n"
    if prefix:
        s += f'snapshot_prefix: "{prefix}/"\n'
    if snapshot:
        s += f"snapshot: {snapshot}\n"
    return s


def _solver(tmp_path, lr, wd, mom, iters, iter_size=1, num=NUM, share=False, snapshot=0, prefix=None):
    from rramsim import caffe
    caffe.set_stream_from_torch()
    caffe.set_random_seed(1701)                                  # Caffe::set_random_seed(this->seed_)
    s = caffe.Solver(solver_proto(lr, wd, mom, iters, iter_size, snapshot, prefix),
                     net_proto(_list_file(tmp_path), num // iter_size, share))
    return s


def _ip_params(s):
    """(weights[D], bias[1]) of layer 'innerprod' (learnable params 0 and 1;
    with sharing, innerprod2's params alias these)."""
    ps = s.net.params()
    return ps[0]["data"].cpu().numpy().astype(np.float64), ps[1]["data"].cpu().numpy().astype(np.float64)


def compute_least_squares_update(s, lr, wd, mom, num):
    """ComputeLeastSquaresUpdate (:224-347) for the SGD solver: one Forward
    for the next batch, then the analytic update from the net's own state."""
    net = s.net
    net.forward()
    X = net.blob("data").cpu().numpy().astype(np.float64).reshape(num, D)
    y = net.blob("targets").cpu().numpy().astype(np.float64).reshape(num)
    w, b = _ip_params(s)
    hist = s.history()
    assert len(hist) == 2                                         # 1 blob for weights, 1 for bias (:292)
    h = np.concatenate([hist[0].cpu().numpy(), hist[1].cpu().numpy()]).astype(np.float64)
    Xa = np.concatenate([X, np.ones((num, 1))], axis=1)
    wa = np.concatenate([w, b])
    grad = (Xa.T @ (Xa @ wa) - Xa.T @ y) / num + wd * wa
    update = lr * grad + mom * h
    return wa - update, update


def _near(expected, got):
    margin = np.maximum(K_MIN_PRECISION, K_PRECISION * np.minimum(np.abs(expected), np.abs(got)))
    bad = np.abs(expected - got) > margin
    assert not bad.any(), (np.flatnonzero(bad)[:8], expected[bad][:8], got[bad][:8])


def check_least_squares_update(s, expected_params, expected_update):
    """CheckLeastSquaresUpdate (:349-397): updated weights and bias, then the
    solver's history (== the last update value for SGD)."""
    w, b = _ip_params(s)
    _near(expected_params, np.concatenate([w, b]))
    hist = s.history()
    h = np.concatenate([hist[0].cpu().numpy(), hist[1].cpu().numpy()]).astype(np.float64)
    _near(expected_update, h)


def least_squares_case(tmp_path, lr=1.0, wd=0.0, mom=0.0, iter_to_check=0, share=False):
    """TestLeastSquaresUpdate (:453-488), devices = 1."""
    s = _solver(tmp_path, lr, wd, mom, iter_to_check, share=share)
    s.step(iter_to_check)
    exp_p, exp_u = compute_least_squares_update(s, lr, wd, mom, NUM)
    s.close()
    s = _solver(tmp_path, lr, wd, mom, iter_to_check + 1, share=share)
    s.step(iter_to_check + 1)
    check_least_squares_update(s, exp_p, exp_u)
    s.close()


def test_hdf5_data_layer_reads_solver_data(device, tmp_path):
    """HDF5Data tops are the file's datasets, batch_size rows per Forward,
    cycling (hdf5_data_layer.cu:17-46): two forwards cover rows 0-3, 4-7."""
    import sys
    sys.path.insert(0, str(ROOT / "tests"))
    from test_hdf5 import H5 as H5Reader
    h = H5Reader()
    data, targets = h.read(H5, "data"), h.read(H5, "targets")
    assert data.shape == (8, 3, 10, 10) and targets.shape == (8, 1)
    from rramsim import caffe
    caffe.set_stream_from_torch()
    net = caffe.Net(net_proto(_list_file(tmp_path), NUM), "train")
    for it in range(3):
        net.forward()
        rows = slice(4 * (it % 2), 4 * (it % 2) + 4)
        assert np.array_equal(net.blob("data").cpu().numpy(), data[rows])
        assert np.array_equal(net.blob("targets").cpu().numpy(), targets[rows])
    net.close()


def test_euclidean_loss_forward_backward(device, tmp_path):
    """EuclideanLoss (euclidean_loss_layer.cu:9-38) on the reference data:
    loss = ||Xw + b - y||^2 / (2n); d loss / d w = X^T (Xw + b - y) / n."""
    s = _solver(tmp_path, 1.0, 0.0, 0.0, 1)
    net = s.net
    net.clear_param_diffs()
    loss = net.forward()
    net.backward()
    X = net.blob("data").cpu().numpy().astype(np.float64).reshape(NUM, D)
    y = net.blob("targets").cpu().numpy().astype(np.float64).reshape(NUM)
    w, b = _ip_params(s)
    r = X @ w + b - y
    assert abs(loss - (r @ r) / NUM / 2) <= 1e-5 * max(1.0, abs(loss))
    ps = net.params()
    np.testing.assert_allclose(ps[0]["diff"].cpu().numpy(), X.T @ r / NUM, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(ps[1]["diff"].cpu().numpy(), [r.sum() / NUM], rtol=1e-4, atol=1e-5)
    s.close()


def test_least_squares_update(device, tmp_path):                       # :574-576
    least_squares_case(tmp_path)


def test_least_squares_update_lr_one_hundredth(device, tmp_path):      # :578-582
    least_squares_case(tmp_path, lr=0.01)


@pytest.mark.parametrize("iters", [1, 4])
def test_least_squares_update_with_weight_decay(device, tmp_path, iters):  # :584-604
    for i in range(iters + 1):
        least_squares_case(tmp_path, 0.01, 0.5, 0.0, i)


@pytest.mark.parametrize("iters", [1, 4])
def test_least_squares_update_with_momentum(device, tmp_path, iters):  # :606-626
    for i in range(iters + 1):
        least_squares_case(tmp_path, 0.01, 0.0, 0.5, i)


@pytest.mark.parametrize("share", [False, True])
def test_least_squares_update_with_everything(device, tmp_path, share):  # :628-649
    for i in range(5):
        least_squares_case(tmp_path, 0.01, 0.5, 0.5, i, share=share)


@pytest.mark.parametrize("share", [False, True])
def test_least_squares_update_with_everything_accum(device, tmp_path, share):  # :651-672
    """CheckAccumulation (:399-436): 4 iterations at batch 4 == 4 iterations
    of iter_size 2 at batch 2 (gradients accumulated, then normalised)."""
    lr, wd, mom, iters = 0.01, 0.5, 0.9, 4
    s = _solver(tmp_path, lr, wd, mom, iters, share=share)
    s.step(iters)
    ref = np.concatenate(_ip_params(s))
    s.close()
    s = _solver(tmp_path, lr, wd, mom, iters, iter_size=2, share=share)
    s.step(iters)
    _near(ref, np.concatenate(_ip_params(s)))
    s.close()


@pytest.mark.parametrize("share", [False, True])
def test_snapshot(device, tmp_path, share):                            # :674-695, TestSnapshot :490-558
    lr, wd, mom = 0.01, 0.5, 0.9
    for k in range(1, 5):
        s = _solver(tmp_path, lr, wd, mom, 2 * k, share=share)
        s.step(2 * k)
        ref_p = [(p["data"].cpu().numpy().copy(), p["diff"].cpu().numpy().copy()) for p in s.net.params()]
        ref_h = [h.cpu().numpy().copy() for h in s.history()]
        s.close()
        prefix = Path(tmp_path) / f"snap{k}{int(share)}"
        prefix.mkdir()
        s = _solver(tmp_path, lr, wd, mom, k, share=share, snapshot=k, prefix=str(prefix))
        s.step(k)
        s.close()
        state = prefix / f"_iter_{k}.solverstate"
        assert state.exists(), list(prefix.iterdir())
        s = _solver(tmp_path, lr, wd, mom, 2 * k, share=share)
        s.restore(str(state))
        for _ in range(s.iter):                                     # advance the data layer (:188-190)
            s.net.forward()
        s.solve()
        for (d0, g0), p in zip(ref_p, s.net.params()):
            assert np.array_equal(d0.view(np.uint32), p["data"].cpu().numpy().view(np.uint32))
            assert np.array_equal(g0.view(np.uint32), p["diff"].cpu().numpy().view(np.uint32))
        for h0, h in zip(ref_h, s.history()):
            assert np.array_equal(h0.view(np.uint32), h.cpu().numpy().view(np.uint32))
        s.close()


# ------------------------------------------------ multi-device (:456-486)
def _free_port():
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    p = sk.getsockname()[1]
    sk.close()
    return p


def _dp_worker(rank, world, port, backend, list_file, cases, q, shard=False):
    import sys
    sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = None
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    elif backend == "native":      # the C++ host's RCCL communicator; gloo only hands out its id
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from rramsim import caffe
        comm = caffe.Comm(rank, world)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    from rramsim.parallel import DataParallelSolver
    out = []
    for lr, wd, mom, iters in cases:
        dp = DataParallelSolver(solver_proto(lr, wd, mom, iters), net_proto(list_file, NUM), seed=1701,
                                shard_hdf5=shard, comm=comm)
        dp.step(iters)
        torch.cuda.synchronize()
        ps = dp.solver.net.params()
        hist = dp.solver.history()
        out.append((np.concatenate([ps[0]["data"].cpu().numpy(), ps[1]["data"].cpu().numpy()]),
                    np.concatenate([hist[0].cpu().numpy(), hist[1].cpu().numpy()]), dp.allreduce_calls))
        dp.close()
    q.put((rank, out))
    dist.barrier()
    if comm is not None:
        comm.close()
    dist.destroy_process_group()


def _run_dp(world, backend, list_file, cases, shard=False):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dp_worker, args=(r, world, port, backend, list_file, cases, q, shard))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda t: t[0])
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def _multi_device_expected(tmp_path, cases, devices):
    """The single-device half of TestLeastSquaresUpdate for `devices` devices:
    num = kNum * devices on one device, K iterations, analytic (K+1)th update."""
    exp = []
    for lr, wd, mom, iters in cases:
        s = _solver(tmp_path, lr, wd, mom, iters - 1, num=NUM * devices)
        s.step(iters - 1)
        exp.append(compute_least_squares_update(s, lr, wd, mom, NUM * devices))
        s.close()
    return exp


def test_least_squares_update_two_ranks(device, tmp_path):
    """devices = 2 with this fork's data semantics: under its P2PSync every
    worker's HDF5Data layer reads its own stream from row 0 (parallel.cpp:
    201-284; hdf5_data_layer.cpp:128-157 has no Skip), so 2 ranks at batch 4
    see the same 4 rows and their averaged gradient is the single-device
    gradient of those rows: 2 data-parallel ranks for K+1 iterations must land
    on the analytic (K+1)th update of one process at batch 4 — for every K of
    the "everything" case, and the ranks stay bitwise identical.  (The
    reference test's own num = kNum x devices comparison, :465-487, needs
    constant data under these semantics; the row split that makes it hold on
    solver_data.h5 is Caffe 1.0's Skip, the opt-in case below.)"""
    cases = [(0.01, 0.5, 0.5, k + 1) for k in range(3)]
    exp = _multi_device_expected(tmp_path, cases, 1)
    res = _run_dp(2, "gloo", _list_file(tmp_path), cases)
    for (ep, eu), (p0, h0, n0), (p1, h1, n1) in zip(exp, res[0][1], res[1][1]):
        _near(ep, p0.astype(np.float64))
        _near(eu, h0.astype(np.float64))
        assert np.array_equal(p0.view(np.uint32), p1.view(np.uint32))
        assert n0 == n1 > 0


def test_least_squares_update_two_ranks_row_split(device, tmp_path):
    """devices = 2 (:465-487) with the opt-in row split (DataParallelSolver
    shard_hdf5=True, Caffe 1.0's HDF5DataLayer::Skip: rank r reads rows r,
    r+2, ...): one process at batch 8 for K iterations, the analytic (K+1)th
    update, then 2 ranks at batch 4 each for K+1 iterations must land on it."""
    cases = [(0.01, 0.5, 0.5, k + 1) for k in range(3)]
    exp = _multi_device_expected(tmp_path, cases, 2)
    res = _run_dp(2, "gloo", _list_file(tmp_path), cases, shard=True)
    for (ep, eu), (p0, h0, n0), (p1, h1, n1) in zip(exp, res[0][1], res[1][1]):
        _near(ep, p0.astype(np.float64))
        _near(eu, h0.astype(np.float64))
        assert np.array_equal(p0.view(np.uint32), p1.view(np.uint32))
        assert n0 == n1 > 0


@pytest.mark.parametrize("backend", ["nccl", "native"])
def test_least_squares_update_rccl_world1(device, tmp_path, backend):
    """The RCCL code paths in a real run, world size 1 on this box's GPU, the
    devices = 1 case of the everything test: torch's (init_process_group
    ("nccl", device_id=...), DataParallelSolver's torch all-reduce) and the
    C++ host's own (caffe.Comm + the native P2PSync, host/parallel.cpp)."""
    cases = [(0.01, 0.5, 0.5, k + 1) for k in range(2)]
    exp = _multi_device_expected(tmp_path, cases, 1)
    res = _run_dp(1, backend, _list_file(tmp_path), cases)
    for (ep, eu), (p0, h0, n0) in zip(exp, res[0][1]):
        _near(ep, p0.astype(np.float64))
        _near(eu, h0.astype(np.float64))
        assert n0 > 0
