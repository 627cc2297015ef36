"""CPU tests of the multi-process path with the gloo backend (world_size 2):
map sharding, gradient averaging (the RCCL all-reduce's arithmetic) and the
statistics all-reduce used by bench.py / the Monte-Carlo driver."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rramsim.parallel import allreduce_stats, average_gradients, shard_maps
    g = torch.full((1000,), float(rank + 1))
    average_gradients(g, world)
    st = allreduce_stats([rank + 0.5, 2.0], "cpu")
    maps = shard_maps(10, rank, world)
    q.put((rank, float(g[0]), st, maps))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gradient_average_and_stats():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1] == 1.5                 # (1 + 2) / 2
    assert res[0][2] == res[1][2] == [2.0, 4.0]          # (0.5 + 1.5), (2 + 2)
    assert res[0][3] == [0, 2, 4, 6, 8] and res[1][3] == [1, 3, 5, 7, 9]


def test_shard_maps_partition():
    from rramsim.parallel import shard_maps
    for world in (1, 2, 4, 8):
        allm = sorted(m for r in range(world) for m in shard_maps(37, r, world))
        assert allm == list(range(37))
