"""Multi-GPU: one process per GPU, torch.distributed over RCCL (xGMI).

Replaces the reference's P2PSync (src/caffe/parallel.cpp:201-437): instead of
a thread per GPU with a peer-to-peer tree broadcast of parameters and tree
reduction of gradients, every rank runs the same deterministic solver on its
own synthetic shard of data; after backward the flat fp32 gradient buffer
(every learnable param aliased into one allocation, the GPUParams layout of
parallel.cpp:25-115) is summed with ONE RCCL all-reduce and scaled by 1/N
(parallel.cpp:377).  The fault state is replicated with identical seeds, so
every rank's Fail() produces the same weights the reference's root-only Fail +
next-iteration broadcast would.

Monte-Carlo inference shards fault maps: map m runs on rank m mod N; the only
collective is the final all-reduce of the statistics vector.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional


def world_info():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def shard_maps(total_maps: int, rank: int, world: int) -> List[int]:
    """Maps owned by `rank` (m mod world == rank)."""
    return list(range(rank, total_maps, world))


def average_gradients(flat, world: int, group=None):
    """Sum-all-reduce the flat gradient buffer and scale by 1/world."""
    import torch.distributed as dist
    if world > 1:
        dist.all_reduce(flat, group=group)
        flat.mul_(1.0 / world)


def allreduce_stats(values: List[float], device, group=None) -> List[float]:
    """One all-reduce (sum, fp64) of a small statistics vector."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, group=group)
    return t.tolist()


class DataParallelSolver:
    """Fault-aware data-parallel SGD (C4) on top of caffe.Solver."""

    def __init__(self, solver_prototxt: str, net_prototxt: str, options: Optional[Dict] = None, seed: int = 1701,
                 group=None, log=None):
        import torch
        import torch.distributed as dist

        from . import caffe
        self.rank, self.world, local = world_info()
        if dist.is_available() and dist.is_initialized():
            self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.group = group
        caffe.set_stream_from_torch()
        caffe.set_random_seed(seed)            # identical weights and fault maps on every rank
        opts = dict(options or {})
        opts["data_seed"] = self.rank           # a different synthetic data shard per rank
        self.solver = caffe.Solver(solver_prototxt, net_prototxt, opts, log=log if self.rank == 0 else None)
        net = self.solver.net
        n = net.flat_param_count()
        dev = torch.device("cuda", torch.cuda.current_device())
        self.flat_data = torch.empty(n, dtype=torch.float32, device=dev)
        self.flat_diff = torch.empty(n, dtype=torch.float32, device=dev)
        net.alias_flat_params(self.flat_data, self.flat_diff)
        if self.world > 1:
            dist.broadcast(self.flat_data, 0, group=group)    # on_start broadcast (parallel.cpp:286-322)
        self.solver.set_gradient_callback(self._on_gradients_ready)
        self.allreduce_calls = 0

    def _on_gradients_ready(self):
        average_gradients(self.flat_diff, self.world, self.group)
        self.allreduce_calls += 1

    def step(self, iters: int):
        self.solver.step(iters)

    @property
    def num_params(self) -> int:
        return self.flat_data.numel()

    def close(self):
        self.solver.close()
