"""Multi-GPU: one process per GPU over RCCL (xGMI).

Two carriers for the same arithmetic: the C++ host's own RCCL communicator
(`caffe.Comm` + `caffe.P2PSync`, host/parallel.cpp: the product path a C or
C++ caller of librram_caffe.so gets, and what bench.py uses on GPUs), and
torch.distributed (gloo: the CPU / shared-GPU rehearsal backend of the tests).

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
import re
from typing import Dict, List, Optional


# The job's RCCL communicator of the C++ host (caffe.Comm), when the caller
# set one: the statistics / timing collectives below and DataParallelSolver's
# default then run on it; unset, they run on torch.distributed (gloo rehearsal).
_COMM = None


def set_comm(comm) -> None:
    global _COMM
    _COMM = comm


def get_comm():
    return _COMM


def _dist_on() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def barrier() -> None:
    if _COMM is not None:
        _COMM.barrier()
    elif _dist_on():
        import torch.distributed as dist
        dist.barrier()


def allreduce_max(x: float, device) -> float:
    """max over ranks of one host value (the bench's max-over-ranks time)."""
    if _COMM is not None:
        return _COMM.allreduce_host([float(x)], "max")[0]
    if not _dist_on():
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def world_info():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def shard_maps(total_maps: int, rank: int, world: int) -> List[int]:
    """Maps owned by `rank` (m mod world == rank)."""
    return list(range(rank, total_maps, world))


def average_gradients(flat, world: int, group=None):
    """Sum-all-reduce the flat gradient buffer and scale by 1/world.  With a
    process group of one rank the all-reduce still runs (the collective path
    is the one a multi-GPU job takes; the sum of one rank is exact)."""
    import torch.distributed as dist
    if world > 1 or (dist.is_available() and dist.is_initialized()):
        dist.all_reduce(flat, group=group)
    if world > 1:
        flat.mul_(1.0 / world)


def plan_buckets(layer_ranges: List[List[tuple]], n_layers: int, bucket_elems: int) -> Dict[int, tuple]:
    """Bucketed gradient all-reduce schedule for backward order.

    layer_ranges[i] lists the [begin, end) flat-buffer ranges of layer i's
    learnable params; the flat buffer holds them in forward layer order
    (Net::alias_flat_params, the GPUParams layout of parallel.cpp:25-115), so
    after layers n-1 ... i have run backward the final gradients form one
    suffix [lo, n) of the buffer.  Returns {layer index: (begin, end)}: after
    that layer's Backward, all-reduce flat[begin:end].  Each bucket holds at
    least bucket_elems elements (except the last, which on_gradients_ready
    launches for whatever is left, so it is not in the plan).  Requires every
    layer's ranges to be contiguous with its neighbours' (no shared params)."""
    plan = {}
    hi = None            # end of the not-yet-reduced suffix
    lo = None
    for i in range(n_layers - 1, -1, -1):
        rs = layer_ranges[i] if i < len(layer_ranges) else []
        if not rs:
            continue
        b, e = min(r[0] for r in rs), max(r[1] for r in rs)
        if hi is None:
            hi = e
        lo = b if lo is None else min(lo, b)
        if hi - lo >= bucket_elems and i > 0:
            plan[i] = (lo, hi)
            hi = lo
            lo = None
    return plan


def allreduce_stats(values: List[float], device, group=None) -> List[float]:
    """One all-reduce (sum, fp64) of a small statistics vector."""
    if _COMM is not None:
        return _COMM.allreduce_host([float(v) for v in values], "sum")
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, group=group)
    return t.tolist()


class DataParallelSolver:
    """Fault-aware data-parallel SGD (C4) on top of caffe.Solver."""

    def __init__(self, solver_prototxt: str, net_prototxt: str, options: Optional[Dict] = None, seed: int = 1701,
                 group=None, log=None, overlap: bool = False, bucket_mb: float = 4.0, shard_hdf5: bool = False,
                 comm="auto"):
        """comm: a caffe.Comm -> the native P2PSync (host/parallel.cpp, RCCL
        from the C++ host); None -> torch.distributed on `group` (gloo
        rehearsal); "auto" -> the communicator set_comm() installed, else None."""
        if isinstance(comm, str):
            comm = _COMM
        import torch
        import torch.distributed as dist

        from . import caffe
        self.rank, self.world, local = world_info()
        if comm is not None:
            self.rank, self.world = comm.rank, comm.world
        elif dist.is_available() and dist.is_initialized():
            self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.group = group
        self.comm = comm
        self.sync = None
        caffe.set_stream_from_torch()
        caffe.set_random_seed(seed)            # identical weights and fault maps on every rank
        opts = dict(options or {})
        opts["data_seed"] = self.rank           # a different synthetic data shard per rank
        # HDF5Data: by default every rank reads every row from row 0, as each
        # P2PSync worker's own data layer does in the reference (parallel.cpp:
        # 201-284; its hdf5_data_layer.cpp:128-157 has no Skip).  shard_hdf5
        # opts into Caffe 1.0's HDF5DataLayer::Skip row split instead (rank r
        # reads rows r, r + N, ...): a deliberate divergence, off by default.
        if shard_hdf5:
            opts["solver_rank"] = self.rank
            opts["solver_count"] = self.world
        self.solver = caffe.Solver(solver_prototxt, net_prototxt, opts, log=log if self.rank == 0 else None)
        m = re.search(r"^\s*iter_size\s*:\s*(\d+)", solver_prototxt, re.M)
        if comm is not None:
            # the C++ P2PSync: broadcast from rank 0 now, all-reduce + 1/N inside step()
            self.sync = caffe.P2PSync(self.solver, comm, bucket_mb=bucket_mb, overlap=overlap)
            flat = self.solver.flat_params()
            assert flat is not None, "the native P2PSync needs the solver's flat parameter buffers"
            self.flat_data, self.flat_diff = flat
            self.overlap = self.sync.info()["buckets"] > 0
            self.allreduce_calls = self.bucket_calls = 0
            return
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
        self.bucket_calls = 0
        self._pending = []
        self._plan = {}
        self._reduced_lo = n
        # iter_size > 1 runs several backward passes per update: only the last
        # one holds the final gradients, so the per-layer buckets stay off
        self.overlap = bool(overlap) and self.world > 1 and not (m and int(m.group(1)) > 1)
        if self.overlap:
            self._plan = self._make_plan(net, int(bucket_mb * (1 << 20)) // 4)
            if self._plan:
                self.solver.set_backward_callback(self._on_layer_backward)
            else:
                self.overlap = False

    def _make_plan(self, net, bucket_elems):
        base = self.flat_data.data_ptr()
        params = net.params()
        ranges, k = [], 0
        for _name, _typ, npar in net.layers():
            rs = []
            for p in params[k:k + npar]:
                b = (p["data"].data_ptr() - base) // 4
                rs.append((b, b + p["data"].numel()))
            ranges.append(rs)
            k += npar
        if k != len(params):          # shared params: the suffix property does not hold
            return {}
        return plan_buckets(ranges, len(ranges), bucket_elems)

    def _on_layer_backward(self, layer):
        # gradients of layers >= `layer` are final: reduce this bucket on the
        # collective stream while backward continues on the compute stream
        import torch.distributed as dist
        r = self._plan.get(layer)
        if r is None:
            return
        b, e = r
        self._pending.append(dist.all_reduce(self.flat_diff[b:e], group=self.group, async_op=True))
        self._reduced_lo = b
        self.bucket_calls += 1

    def _on_gradients_ready(self):
        if self.overlap:
            import torch.distributed as dist
            if self._reduced_lo > 0:
                self._pending.append(dist.all_reduce(self.flat_diff[:self._reduced_lo], group=self.group,
                                                     async_op=True))
                self.bucket_calls += 1
            for w in self._pending:
                w.wait()              # the compute stream waits for the collective stream
            self._pending = []
            self._reduced_lo = self.flat_diff.numel()
            self.flat_diff.mul_(1.0 / self.world)
        else:
            average_gradients(self.flat_diff, self.world, self.group)
        self.allreduce_calls += 1

    def step(self, iters: int):
        self.solver.step(iters)
        if self.sync is not None:
            i = self.sync.info()
            self.allreduce_calls, self.bucket_calls = i["allreduce_calls"], i["bucket_calls"]

    @property
    def num_params(self) -> int:
        return self.flat_data.numel()

    def close(self):
        if self.sync is not None:
            self.sync.close()
        self.solver.close()
