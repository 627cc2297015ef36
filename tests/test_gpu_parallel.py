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
