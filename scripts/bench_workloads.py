"""The non-headline BASELINE.json configs as bench.py workloads
(`python bench.py --workload NAME`); each prints one JSON line like the
headline.  Same contract: W untimed warmup steps, K timed steps bracketed by
barrier + synchronize, max over ranks, whole-job throughput.

  cifar10_quick_mc   C2: CIFAR-10 quick, conductance quantisation + lognormal
                     variation, Monte-Carlo fault maps (1 map = one 100-image batch)
  cifar10_full_train C4: CIFAR-10 full fault-aware training (failure_pattern
                     mean 5e6 / std 1.5e6 / prob 5, threshold strategy), data-parallel
                     RCCL gradient all-reduce, fused update+fail tail
  googlenet_sweep    C5: GoogLeNet b256 inference sweep over fault rate
                     0.1 .. 10 %, per-layer SA0/SA1 (neg/zero/pos) ratios
  lenet_train        C1's net (LeNet, stuck-at faults) trained on the GPU
"""
from __future__ import annotations

import math
import time

MFMA_F32_PEAK_TFLOPS = 157.3


def _timed(world, dev, fn, steps, warmup):
    import torch
    import torch.distributed as dist
    for i in range(warmup):
        fn(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(warmup + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _base(metric, unit, value, world, args, el, dtype="f32", **cfg):
    return {"metric": metric, "value": round(value, 3), "unit": unit, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": "synthetic", "config": cfg}


def run_workload(args, world, rank, dev):
    import torch
    import torch.distributed as dist
    from rramsim import caffe, make_inject_cfg, models
    from rramsim.parallel import DataParallelSolver, allreduce_stats

    if args.workload == "cifar10_quick_mc":
        batch = 100
        net = caffe.Net(models.cifar10_quick(test_batch=batch), "test", models.net_options("cifar10_quick"))
        # conductance-quantised (16 levels over the blob's |w| range) + lognormal sigma 0.1, 1 % stuck-at
        fps = net.failure_params()
        cfgs = []
        for f in fps:
            gmax = float(f["data"].abs().max().item()) or 1.0
            cfgs.append(make_inject_cfg(0.01, 10, 20, 10, quant_levels=16, g_max=gmax, var_sigma=0.1,
                                        stuck_scale=gmax))
        mc = caffe.MonteCarlo(net, cfgs, seed=args.seed, max_maps=args.steps + args.warmup + 8)
        maps_per_step = 10
        el = _timed(world, dev, lambda i: mc.run((rank + world * i) * maps_per_step, maps_per_step),
                    args.steps, args.warmup)
        st = mc.stats()
        tot = allreduce_stats(st["sums"] + [st["maps"]], dev)
        n_maps = world * args.steps * maps_per_step
        res = _base("Monte Carlo fault maps/sec, CIFAR-10 quick (quantised + lognormal)", "maps/s", n_maps / el,
                    world, args, el, workload="cifar10_quick_mc_quant16_lognormal0.1", model="CIFAR10_quick",
                    global_batch=batch * world, maps_per_step=maps_per_step * world, p_fault=0.01)
        res["images_per_s"] = round(n_maps * batch / el, 1)
        res["mc_mean_outputs"] = [x / max(tot[-1], 1) for x in tot[:-1]]
        mc.close()
        net.close()
        return res

    if args.workload in ("cifar10_full_train", "lenet_train"):
        if args.workload == "cifar10_full_train":
            batch, net_txt, opts = 100, models.cifar10_full(train_batch=100, test_batch=100), models.net_options("cifar10_full")
            # run_different_th.sh:3-10: mean 5e6, std 1.5e6, prob 5 -> (5, 90, 5), threshold strategy
            sp = models.solver(base_lr=0.001, momentum=0.9, weight_decay=0.004, max_iter=100000,
                               failure_mean=5e6, failure_std=1.5e6, failure_prob=(5, 90, 5), threshold=0.001)
        else:
            batch, net_txt, opts = 64, models.lenet(train_batch=64), models.net_options("lenet")
            sp = models.solver(base_lr=0.01, momentum=0.9, weight_decay=0.0005, lr_policy="inv", gamma=0.0001,
                               power=0.75, max_iter=100000, failure_mean=5e3, failure_std=1e3,
                               failure_prob=(10, 20, 10))
        opts = dict(opts, fused_update=True)
        dp = DataParallelSolver(sp, net_txt, opts, seed=args.seed)
        el = _timed(world, dev, lambda i: dp.step(1), args.steps, args.warmup)
        res = _base(f"fault-aware training images/sec, {args.workload}", "images/s",
                    world * args.steps * batch / el, world, args, el, workload=args.workload,
                    model=args.workload.split("_")[0], global_batch=batch * world,
                    parallelism=f"dp{world} (RCCL all-reduce of {dp.num_params} fp32 grads)")
        res["broken_cells"] = sum(dp.solver.broken_counts())
        dp.close()
        return res

    if args.workload == "googlenet_sweep":
        batch = args.batch
        net = caffe.Net(models.googlenet(test_batch=batch), "test", models.net_options("googlenet"))
        rates = [0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.10]
        nblobs = len(net.failure_params())
        # per-layer SA ratios: classifier weights lean SA0 (zero), aux-heads lean SA1 (+-1)
        def cfgs_for(p):
            out = []
            for i in range(nblobs):
                neg, zero, pos = (5, 90, 5) if i >= nblobs - 2 else (20, 60, 20)
                out.append(make_inject_cfg(p, neg, zero, pos))
            return out
        mcs = [caffe.MonteCarlo(net, cfgs_for(p), seed=args.seed + k, max_maps=args.steps + args.warmup + 8)
               for k, p in enumerate(rates)]

        def step(i):
            for mc in mcs:                       # one map per fault rate per step
                mc.run(rank + world * i, 1)
        el = _timed(world, dev, step, args.steps, args.warmup)
        sweep = []
        for p, mc in zip(rates, mcs):
            st = mc.stats()
            tot = allreduce_stats(st["sums"] + [st["maps"]], dev)
            sweep.append({"p_fault": p, "mean_outputs": [x / max(tot[-1], 1) for x in tot[:-1]]})
        n_img = world * args.steps * len(rates) * batch
        res = _base("Monte Carlo fault-map inferences/sec, GoogLeNet fault-rate sweep", "images/s", n_img / el,
                    world, args, el, workload="googlenet_sweep_0.1-10pct", model="GoogLeNet (train_val TEST)",
                    global_batch=batch * world, rates=rates)
        res["sweep"] = sweep
        for mc in mcs:
            mc.close()
        net.close()
        return res
    raise ValueError(args.workload)
