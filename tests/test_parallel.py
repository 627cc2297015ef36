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


def test_plan_buckets_suffixes_in_backward_order():
    """The bucket plan covers the flat gradient buffer as disjoint suffix
    slices in backward order; the remainder [0, last lo) is left to
    on_gradients_ready; paramless layers are skipped."""
    from rramsim.parallel import plan_buckets
    # layers: data, conv1(w,b), pool, conv2(w,b), ip1(w,b), relu, ip2(w,b), loss
    sizes = {1: (500, 20), 3: (25000, 50), 4: (400000, 500), 6: (5000, 10)}
    ranges, off = [], 0
    for i in range(8):
        rs = []
        for n in sizes.get(i, ()):
            rs.append((off, off + n))
            off += n
        ranges.append(rs)
    total = off
    for be in (1, 1000, 30000, 10 ** 9):
        plan = plan_buckets(ranges, 8, be)
        hi = total
        for layer in sorted(plan, reverse=True):
            b, e = plan[layer]
            assert e == hi and b < e and (e - b >= be)
            assert b == min(r[0] for r in ranges[layer])     # bucket ends at this layer's first param
            hi = b
        assert hi >= 0 and 0 not in plan                      # layer 0's remainder goes at gradients-ready
    assert plan_buckets(ranges, 8, 10 ** 9) == {}
    off = {1: 0, 3: 520, 4: 25570, 6: 426070}
    p1 = plan_buckets(ranges, 8, 1)                        # every param layer its own bucket
    assert p1 == {6: (426070, total), 4: (25570, 426070), 3: (520, 25570), 1: (0, 520)}
    assert off[6] == 426070
    p2 = plan_buckets(ranges, 8, 30000)                    # small tail layers merge upward
    assert p2 == {4: (25570, total)}                       # [0, 25570) is the gradients-ready remainder


def _bucket_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rramsim.parallel import average_gradients, plan_buckets
    g = torch.arange(10_000, dtype=torch.float32) * (rank + 1) / 7.0
    ref = g.clone()
    average_gradients(ref, world)
    ranges = [[], [(0, 3000)], [], [(3000, 9000), (9000, 9100)], [(9100, 10_000)]]
    plan = plan_buckets(ranges, len(ranges), 2000)
    works, lo = [], g.numel()
    for layer in range(len(ranges) - 1, -1, -1):            # backward order
        if layer in plan:
            b, e = plan[layer]
            works.append(dist.all_reduce(g[b:e], async_op=True))
            lo = b
    if lo > 0:
        works.append(dist.all_reduce(g[:lo], async_op=True))
    for w in works:
        w.wait()
    g.mul_(1.0 / world)
    q.put((rank, bool(torch.equal(g, ref)), sorted(plan.items())))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_bucketed_allreduce_equals_flat():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] and res[1][1]
    assert res[0][2] == [(1, (0, 3000)), (3, (3000, 10_000))]


def test_native_plan_buckets_matches_python_plan():
    """The C++ P2PSync's bucket plan (host/parallel.cpp plan_buckets, exposed
    host-only as rram_dp_plan_buckets) is the Python rehearsal's plan on the
    LeNet-shaped layout above, on random layouts with paramless layers, and
    refuses layouts whose ranges do not tile the buffer in layer order (shared
    params: the suffix property fails)."""
    import random
    from rramsim import caffe
    from rramsim.parallel import plan_buckets
    sizes = {1: (500, 20), 3: (25000, 50), 4: (400000, 500), 6: (5000, 10)}
    rng = random.Random(5)
    layouts = []
    ranges, off = [], 0
    for i in range(8):
        rs = []
        for n in sizes.get(i, ()):
            rs.append((off, off + n))
            off += n
        ranges.append(rs)
    layouts.append(ranges)
    for _ in range(40):
        ranges, off = [], 0
        for i in range(rng.randint(1, 30)):
            rs = []
            for _ in range(rng.choice((0, 0, 1, 2, 3))):
                n = rng.randint(1, 100_000)
                rs.append((off, off + n))
                off += n
            ranges.append(rs)
        layouts.append(ranges)
    for ranges in layouts:
        for be in (1, 1000, 30000, 200_000, 10 ** 9):
            assert caffe.dp_plan_buckets(ranges, be) == plan_buckets(ranges, len(ranges), be), (ranges, be)
    # a param shared by two layers (its range appears twice): no plan
    shared = [[(0, 10)], [(10, 20)], [(0, 10)]]
    assert caffe.dp_plan_buckets(shared, 1) == {}


def test_caffe_signatures_cover_the_header():
    """Every rram_caffe.h entry point, the multi-GPU ones included, has a
    ctypes signature in rramsim.caffe (the Python view is complete)."""
    import re
    from pathlib import Path
    from rramsim import caffe
    text = (Path(__file__).resolve().parents[1] / "include" / "rram_caffe.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(rram_[a-z0-9_]+)\s*\(", text))
    assert {"rram_comm_create", "rram_dp_create", "rram_mc_allreduce_stats"} <= names
    assert sorted(names - set(caffe.SIGNATURES)) == []
