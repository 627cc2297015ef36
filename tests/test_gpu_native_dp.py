"""The data-parallel path of the C++ host (host/parallel.cpp: Comm + P2PSync
over RCCL, include/rram_caffe.h rram_comm_* / rram_dp_*), replacing the
reference's P2PSync (src/caffe/parallel.cpp:201-437; tools/caffe.cpp:247-249).

On this box's one GPU the communicator runs at world size 1: the broadcast,
the per-iteration all-reduce of the flat gradient buffer and the statistics
all-reduce are real RCCL calls made from librram_caffe.so.  Gates: a compiled
C driver (tests/abi_dp.c, built by the Makefile) training C4 (CIFAR-10 full,
fault-aware: fused update + threshold + Fail) and the Python view of the same
native path both give bit-identical weights and broken counts to the torch
path and to a plain solver."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
ABI_DP = ROOT / "rram-caffe-simulation_amd" / "build" / "abi_dp"


def _c4(iters=3):
    from rramsim import models
    net = models.cifar10_full(train_batch=32, test_batch=32)
    sp = models.solver(base_lr=0.001, momentum=0.9, weight_decay=0.004, max_iter=1000,
                       failure_mean=2e3, failure_std=1e3, failure_prob=(5, 90, 5), threshold=0.001)
    opts = dict(models.net_options("cifar10_full"), fused_update=True)
    return sp, net, opts


def _python_dp(comm, iters, overlap=True):
    import torch
    from rramsim.parallel import DataParallelSolver
    sp, net, opts = _c4()
    dp = DataParallelSolver(sp, net, opts, seed=1701, overlap=overlap, comm=comm)
    dp.step(iters)
    torch.cuda.synchronize()
    w = dp.flat_data.cpu().numpy().copy()
    b = dp.solver.broken_counts()
    calls = dp.allreduce_calls
    native = dp.sync is not None
    dp.close()
    return w, b, calls, native


def test_native_p2psync_world1_equals_torch_path(device):
    """Python through the native P2PSync (caffe.Comm at world 1: RCCL from
    the C++ host) == the torch-carried DataParallelSolver == the plain solver,
    bit for bit after 3 fault-aware iterations; one all-reduce per iteration."""
    import torch
    from rramsim import caffe
    w_t, b_t, calls_t, nat_t = _python_dp(None, 3)
    comm = caffe.Comm(0, 1)
    try:
        w_n, b_n, calls_n, nat_n = _python_dp(comm, 3)
    finally:
        comm.close()
    assert nat_n and not nat_t
    assert calls_n == 3
    sp, net, opts = _c4()
    caffe.set_stream_from_torch()
    caffe.set_random_seed(1701)
    s = caffe.Solver(sp, net, dict(opts, data_seed=0))
    s.step(3)
    torch.cuda.synchronize()
    w_ref = s.flat_params()[0].cpu().numpy().copy()
    b_ref = s.broken_counts()
    s.close()
    assert sum(b_ref) > 0                      # faults fired
    assert np.array_equal(w_n.view(np.uint32), w_ref.view(np.uint32))
    assert np.array_equal(w_t.view(np.uint32), w_ref.view(np.uint32))
    assert b_n == b_t == b_ref


def test_abi_dp_c_driver_world1(device, tmp_path):
    """tests/abi_dp.c — a plain-C program linking librram_caffe.so — trains C4
    through rram_comm_create / rram_dp_create at RCCL world 1 and writes its
    weights: bit-identical to the Python native path and the torch path."""
    from rramsim import caffe
    assert ABI_DP.exists(), "build/abi_dp not built (make -C rram-caffe-simulation_amd)"
    sp, net, opts = _c4()
    (tmp_path / "solver.prototxt").write_text(sp)
    (tmp_path / "net.prototxt").write_text(net)
    out = tmp_path / "w.bin"
    r = subprocess.run([str(ABI_DP), str(tmp_path / "solver.prototxt"), str(tmp_path / "net.prototxt"),
                        caffe.options_text(opts).decode(), "3", str(out)],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "world 1" in r.stdout and "allreduce_calls 3" in r.stdout, r.stdout
    w_t, b_t, _, _ = _python_dp(None, 3)
    raw = out.read_bytes()
    w_c = np.frombuffer(raw[:4 * w_t.size], dtype=np.float32)
    b_c = np.frombuffer(raw[4 * w_t.size:], dtype=np.uint64).tolist()
    assert len(raw) == 4 * w_t.size + 8 * len(b_t)
    assert np.array_equal(w_c.view(np.uint32), w_t.view(np.uint32))
    assert b_c == b_t and sum(b_c) > 0


def test_native_mc_stats_allreduce_world1(device):
    """rram_mc_allreduce_stats at world 1 returns the map job's own output
    sums, total broken cells and map count (one RCCL all-reduce), and the
    communicator's host max / barrier run."""
    from rramsim import caffe, make_inject_cfg, models
    caffe.set_stream_from_torch()
    caffe.set_random_seed(1701)
    net = caffe.Net(models.lenet(test_batch=50), "test", models.net_options("lenet"))
    mc = caffe.MonteCarlo(net, make_inject_cfg(0.05), seed=11, max_maps=16)
    mc.run(0, 5)
    st = mc.stats()
    comm = caffe.Comm(0, 1)
    try:
        got = comm.mc_stats(mc)
        assert got == st["sums"] + [float(sum(st["broken"])), float(st["maps"])]
        assert comm.allreduce_host([1.5, -2.0], "max") == [1.5, -2.0]
        comm.barrier()
    finally:
        comm.close()
        mc.close()
        net.close()


def test_native_p2psync_solver_destroyed_first(device):
    """Destroying the solver before its P2PSync detaches the sync (its hooks
    point into the solver): the later rram_dp_destroy only frees the handle,
    rram_dp_info reports the detached state, and a second P2PSync on one
    solver is refused."""
    import ctypes as C
    from rramsim import caffe
    sp, net, opts = _c4()
    caffe.set_stream_from_torch()
    caffe.set_random_seed(1701)
    comm = caffe.Comm(0, 1)
    try:
        s = caffe.Solver(sp, net, opts)
        dp = caffe.P2PSync(s, comm)
        with pytest.raises(Exception):
            caffe.P2PSync(s, comm)                 # one per solver
        s.step(1)
        assert dp.info()["allreduce_calls"] == 1
        s.close()                                  # the solver goes first
        lib = caffe.load()
        a = C.c_longlong()
        assert lib.rram_dp_info(dp.h, C.byref(a), None, None, None) != 0
        dp.close()
    finally:
        comm.close()
