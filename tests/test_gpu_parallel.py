"""Data-parallel fault-aware training on the GPU: two ranks on the box's GPU
(gloo carries the collectives here; the product uses RCCL on 1 GPU per rank).
Each rank trains on a different synthetic shard; after every step the replicas
must hold identical weights and identical fault state (averaged gradients +
replicated deterministic Fail())."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root / "rram-caffe-simulation_amd" / "python"))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rramsim import models
    from rramsim.parallel import DataParallelSolver
    sp = models.solver(base_lr=0.01, momentum=0.9, weight_decay=0.0005, max_iter=10,
                       failure_mean=400.0, failure_std=200.0, threshold=0.0005)
    dp = DataParallelSolver(sp, models.lenet(train_batch=32, test_batch=32), models.net_options("lenet"), seed=7)
    dp.step(3)
    torch.cuda.synchronize()
    w = dp.flat_data.double()
    e = torch.cat([s[0] for s in dp.solver.fail_state()]).double()
    data0 = dp.solver.net.blob("data").sum().item()
    q.put((rank, float(w.sum()), float((w * w).sum()), float(e.sum()), dp.allreduce_calls, data0,
           dp.solver.broken_counts()))
    dist.barrier()
    dp.close()
    dist.destroy_process_group()


def test_two_ranks_stay_identical(device):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    (_, w0, ww0, e0, n0, d0, b0), (_, w1, ww1, e1, n1, d1, b1) = res
    assert n0 == n1 == 3                       # one gradient all-reduce per iteration
    assert d0 != d1                            # different data shards per rank
    assert w0 == w1 and ww0 == ww1             # bitwise-identical replicas
    assert e0 == e1 and b0 == b1               # identical fault state


def _equiv_worker(rank, world, port, q, data, label, overlap):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root / "rram-caffe-simulation_amd" / "python"))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rramsim import models
    from rramsim.parallel import DataParallelSolver
    dp = DataParallelSolver(_equiv_solver(), models.lenet(train_batch=32, test_batch=32),
                            models.net_options("lenet"), seed=7, overlap=overlap, bucket_mb=0.25)
    net = dp.solver.net
    b = data.shape[0] // world
    net.blob("data").copy_(torch.from_numpy(data[rank * b:(rank + 1) * b]).reshape(net.blob("data").shape))
    net.blob("label").copy_(torch.from_numpy(label[rank * b:(rank + 1) * b]))
    dp.step(3)
    torch.cuda.synchronize()
    w = dp.flat_data.cpu().numpy().copy()
    e = torch.cat([s[0] for s in dp.solver.fail_state()]).cpu().numpy().copy()
    q.put((rank, w, e, dp.solver.broken_counts(), dp.allreduce_calls, dp.bucket_calls, dp.overlap))
    dist.barrier()
    dp.close()
    dist.destroy_process_group()


def _equiv_solver():
    from rramsim import models
    return models.solver(base_lr=0.01, momentum=0.9, weight_decay=0.0005, max_iter=10,
                         failure_mean=250.0, failure_std=150.0)


def _run_equiv(data, label, overlap):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_equiv_worker, args=(r, 2, port, q, data, label, overlap)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda t: t[0])
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def test_dp_two_ranks_equal_one_process_double_batch(device):
    """P2PSync semantics (parallel.cpp:324-380: sum of the ranks' gradients,
    scaled by 1/N on the root) make 2 ranks x batch 32 the same SGD as one
    process x batch 64 holding both shards (the reference's multi-GPU solver
    test pattern, test_gradient_based_solver.cpp:191-209,456-486).  After 3
    iterations with stuck-at faults: weights within 1e-6 relative (gradient
    summation order differs), endurance and broken counts bit-exact.  The
    bucketed all-reduce overlapped with backward gives the
    same bits as the single flat all-reduce."""
    import numpy as np
    import torch
    from rramsim import caffe, models
    caffe.set_stream_from_torch()
    caffe.set_random_seed(7)
    s = caffe.Solver(_equiv_solver(), models.lenet(train_batch=64, test_batch=64), models.net_options("lenet"))
    data = s.net.blob("data").cpu().numpy().copy()
    label = s.net.blob("label").cpu().numpy().copy()
    s.step(3)
    torch.cuda.synchronize()
    w_ref = torch.cat([p["data"] for p in s.net.params()]).cpu().numpy()
    e_ref = torch.cat([f[0] for f in s.fail_state()]).cpu().numpy()
    b_ref = s.broken_counts()
    s.close()
    assert sum(b_ref) > 0                                  # faults fired during the 3 steps
    flat = _run_equiv(data, label, overlap=False)
    for rank, w, e, b, calls, bcalls, ov in flat:
        assert calls == 3 and not ov
        np.testing.assert_allclose(w, w_ref, rtol=1e-6, atol=1e-7 * float(np.abs(w_ref).max()))
        assert np.array_equal(e.view(np.uint32), e_ref.view(np.uint32)), rank
        assert b == b_ref
    assert np.array_equal(flat[0][1], flat[1][1])
    over = _run_equiv(data, label, overlap=True)
    for (rank, w, e, b, calls, bcalls, ov), f in zip(over, flat):
        assert ov and calls == 3 and bcalls > 3            # more than one bucket per iteration
        assert np.array_equal(w.view(np.uint32), f[1].view(np.uint32)), rank
        assert np.array_equal(e.view(np.uint32), f[2].view(np.uint32)) and b == f[3]


@pytest.mark.parametrize("workload", ["alexnet_mc", "cifar10_full_train"])
def test_bench_two_ranks_rehearsal(device, workload):
    """bench.py's N > 1 path end to end (torch.distributed.run, 2 ranks, map /
    batch sharding, barrier + max-over-ranks timing, stats all-reduce, the
    overlapped gradient buckets of the training workload) on this box's one
    GPU: RRAM_BENCH_DIST_BACKEND=gloo lets both ranks share it (the driver's
    multi-GPU runs use RCCL, one GPU per rank)."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, RRAM_BENCH_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(root / "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--workload", workload]
    if workload == "alexnet_mc":
        cmd += ["--batch", "64"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(root))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout                     # rank 0 prints exactly one JSON line
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 3 and res["value"] > 0
    if workload == "alexnet_mc":
        assert res["mc_stats"]["maps"] == 6              # 3 maps on each of the 2 ranks
        assert res["config"]["global_batch"] == 128 and res["cpu_baseline"] is None
    else:
        # 89,578 fp32 grads fit one 4 MB bucket: a single all-reduce, no overlap plan
        assert res["config"]["parallelism"].startswith("dp2 (RCCL all-reduce of 89578 fp32 grads")


@pytest.mark.parametrize("workload", ["alexnet_mc", "cifar10_full_train"])
def test_bench_rccl_world1(device, workload):
    """bench.py under torch.distributed.run with the default backend (RCCL):
    world size 1 on this box's GPU runs the C++ host's own RCCL communicator
    (torch.distributed is only the gloo rendezvous that hands out its id):
    the barriers, the stats / max-time all-reduces and (for training) the
    native P2PSync gradient all-reduce — the collectives an 8-GPU job issues
    (replaces parallel.cpp:324-380)."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k != "RRAM_BENCH_DIST_BACKEND"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(root / "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--workload", workload, "--no-cpu-baseline"]
    if workload == "alexnet_mc":
        cmd += ["--batch", "64"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(root))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 1 and res["value"] > 0
    if workload == "alexnet_mc":
        assert res["config"]["parallelism"] == \
            "mc-maps x1 (RCCL stats all-reduce from the C++ host, rram_mc_allreduce_stats)"
        assert res["mc_stats"]["maps"] == 3
    else:
        p = res["config"]["parallelism"]
        assert p.startswith("dp1 (RCCL all-reduce") and "C++ host P2PSync" in p, p
