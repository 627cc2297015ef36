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
  lenet_mc           C1: LeNet stuck-at Monte-Carlo fault maps (1 map = one
                     100-image batch), with the Caffe-CPU-mode restatement
                     (oracle inject + per-image im2col + OpenBLAS sgemm) timed
                     beside it on rank 0 at N = 1
"""
from __future__ import annotations

import math
import os
import time

MFMA_F32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: fp32 MFMA dense
MFMA_X6_PEAK_TFLOPS = 2500.0 / 6  # bf16 dense peak / the bf16x6 engine's 6 products
PEAK_OF_ENGINE = {0: MFMA_F32_PEAK_TFLOPS, 1: MFMA_X6_PEAK_TFLOPS}


def map_statistics(s, s2, n):
    """Mean, sample standard deviation and 95 % CI half-width (normal
    approximation, 1.96 sigma / sqrt(n)) of n per-map values from their sum s
    and sum of squares s2 (all-reduced over ranks by the caller)."""
    nm = max(int(n), 1)
    mean = s / nm
    var = max(s2 / nm - mean * mean, 0.0) * nm / max(nm - 1, 1)
    return dict(mean=mean, std=var ** 0.5, ci95=1.96 * (var / nm) ** 0.5, maps=int(n))


def contraction_roofline(net, passes, lt=None, note=""):
    """Roofline of a net's Convolution / InnerProduct forward contractions
    (the dominant kernels): algorithmic FLOPs per forward pass from
    rram_net_layer_contraction, times from the live hipEvent layer timers of
    the timed region (`lt` = net.layer_times(), `passes` forwards timed); the
    peak is each layer's engine peak (fp32 MFMA 157.3, bf16x6 416.7)."""
    con = net.contractions()
    flops = sum(f for f, e in con.values())
    t_min = sum(f / (PEAK_OF_ENGINE[e] * 1e12) for f, e in con.values())
    peak = flops / t_min / 1e12
    out = {"bound": "mfma", "peak": round(peak, 1), "unit": "TFLOP/s", "traffic": None,
           "algorithmic_flops_per_pass": flops,
           "engines": {"bf16x6": sum(1 for f, e in con.values() if e == 1), "f32": sum(1 for f, e in con.values() if e == 0)},
           "flops_share_bf16x6": round(sum(f for f, e in con.values() if e == 1) / max(flops, 1.0), 3)}
    if lt is not None:
        ms = sum(m for (name, typ, m, cnt) in lt if name in con) / passes
        out.update(achieved=round(flops / (ms * 1e-3) / 1e12, 2), frac=round(flops / (ms * 1e-3) / 1e12 / peak, 4),
                   avg_ms_per_pass=round(ms, 4), kernel="Convolution + InnerProduct forward contractions, live "
                   "hipEvent layer timers over the timed region" + note)
    return out


def mc_cpu_baseline(model_fn, name, batch, cfgs, seed, budget_s=10.0):
    """Caffe CPU mode for an MC workload (oracle/cpu_net.py, TEST
    infrastructure): the map's injection into the faultable blobs through
    the C oracle plus single-image forwards (per-image im2col + OpenBLAS sgemm,
    scalar pool / LRN / ReLU loops) for ~budget_s, extrapolated to one
    `batch`-image map; OpenBLAS on the host's physical cores."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "oracle"))
    import cpu_net
    import oracle
    from rramsim import models
    import os
    ds = tuple(int(v) for v in str(models.net_options(name)["data_shape"]).split(","))
    ocfgs = [oracle.InjectCfg(c.thr_fault, c.thr_neg, c.thr_zero, c.thr_sa1, c.stuck_scale, c.g_max, c.quant_levels,
                              c.var_sigma, c.cell_mode, 0) for c in cfgs]
    # physical cores and the per-GPU CPU share (OMP_NUM_THREADS): the faster is
    # the baseline (OpenBLAS over every core of a shared box can lose on
    # per-image GEMMs), both are reported
    phys = oracle.physical_cores()
    env = os.environ.get("OMP_NUM_THREADS", "")
    share = int(env) if env.isdigit() else 0
    runs = {}
    for th in sorted({phys} | ({share} if 0 < share < phys else set())):
        runs[th] = cpu_net.mc_map_sample(model_fn(test_batch=batch), ds, batch, ocfgs, seed=seed,
                                         budget_s=budget_s / 2, threads=th)
    th = max(runs, key=lambda k: runs[k][0])
    v, meta = runs[th]
    return {"value": round(v, 3), "unit": "images/s", "cores": meta["threads"], "kind": "port",
            "by_threads": {str(k): round(r[0], 3) for k, r in runs.items()},
            "sample": f"1 fault map ({meta['broken']} of {meta['faultable_weights']:,} faultable cells broken by the C "
                      f"oracle in {meta['t_inject'] * 1e3:.1f} ms) + {meta['images']} single-image TEST forwards in "
                      f"Caffe CPU mode ({meta['t_img'] * 1e3:.2f} ms/img; sgemm = {meta['blas']} on {meta['threads']} "
                      f"threads), extrapolated to one {batch}-image map",
            "layer_share": meta["layer_share"]}


def _dist_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def _timed(world, dev, fn, steps, warmup, net=None, block=None):
    """Warmup, then `steps` timed calls bracketed by barrier + synchronize;
    max over ranks.  With `net`, its hipEvent timers run around the
    Convolution / InnerProduct layers during the timed calls only.  With
    `block`, the warmup and the timed steps are one call each, block(n), as
    `caffe train` runs Solver::Step over all its iterations."""
    import torch
    import torch.distributed as dist
    if block is not None:
        fn = None
        if warmup:
            block(warmup)
    for i in range(warmup if fn is not None else 0):
        fn(i)
    torch.cuda.synchronize()
    if net is not None:
        net.layer_times(reset=True)
        net.set_timing(2)
    from rramsim import parallel
    parallel.barrier()        # the C++ host's RCCL communicator when bench.py set one, else torch.distributed
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if block is not None:
        block(steps)
    else:
        for i in range(steps):
            fn(warmup + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if net is not None:
        net.set_timing(0)
    return parallel.allreduce_max(el, dev)


def _base(metric, unit, value, world, args, el, dtype="f32", **cfg):
    return {"metric": metric, "value": round(value, 3), "unit": unit, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": "synthetic", "config": cfg}


def lenet_cpu_baseline(batch, p_fault, seed, budget_s=10.0):
    """Caffe CPU mode for C1 (restated in oracle/): one stuck-at map injected
    into LeNet's 405,510 IP weights by the scalar C oracle, then single-image
    forwards (im2col + sgemm per conv, as conv_layer.cpp:7-27) until the budget
    is spent; images/s extrapolated to one `batch`-image map."""
    import os
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "oracle"))
    import numpy as np
    import oracle
    from rramsim import make_inject_cfg
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("internal_api") == "openblas"]
                      or [1])
    except Exception:  # pragma: no cover
        threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    rng = np.random.default_rng(seed)
    w1 = (rng.standard_normal((20, 1, 5, 5)) * 0.1).astype(np.float32)
    w2 = (rng.standard_normal((50, 20, 5, 5)) * 0.05).astype(np.float32)
    b1, b2 = np.zeros(20, np.float32), np.zeros(50, np.float32)
    fw = {"ip1": (rng.standard_normal((500, 800)) * 0.05).astype(np.float32),
          "ip2": (rng.standard_normal((10, 500)) * 0.05).astype(np.float32)}
    fb = {"ip1": np.zeros(500, np.float32), "ip2": np.zeros(10, np.float32)}
    c = make_inject_cfg(p_fault)
    oc = oracle.InjectCfg(c.thr_fault, c.thr_neg, c.thr_zero, c.thr_sa1, 1.0, 0.0, 0, 0.0, 0, 0)
    t0 = time.perf_counter()
    for lid, k in enumerate(fw):
        fw[k], _ = oracle.inject(fw[k], oc, seed, 0, 2 * lid)
        fb[k], _ = oracle.inject(fb[k], oc, seed, 0, 2 * lid + 1)
    t_inject = time.perf_counter() - t0
    x_all = (rng.integers(0, 256, (batch, 1, 28, 28)) * 0.00390625).astype(np.float32)

    def fwd(x):
        y = oracle.pool(oracle.conv_im2col(x, w1, b1), 2, 2)
        y = oracle.pool(oracle.conv_im2col(y, w2, b2), 2, 2).reshape(x.shape[0], -1)
        y = np.maximum(y @ fw["ip1"].T + fb["ip1"], 0)
        return oracle.softmax(y @ fw["ip2"].T + fb["ip2"])

    n, t1 = 0, time.perf_counter()
    while n < 2 or (time.perf_counter() - t1 < budget_s and n < 200 * batch):
        fwd(x_all[n % batch:n % batch + 1])
        n += 1
    t_img = (time.perf_counter() - t1) / n
    return {"value": round(batch / (t_inject + batch * t_img), 3), "unit": "images/s", "cores": threads,
            "kind": "port",
            "sample": f"1 fault map (C oracle inject of 405,510 IP weights: {t_inject * 1e3:.1f} ms) + {n} "
                      f"single-image LeNet forwards (im2col + OpenBLAS sgemm: {t_img * 1e3:.3f} ms/img), "
                      f"extrapolated to one {batch}-image map"}


def _graph_on():
    """MonteCarlo / Solver hipGraph replay for the launch-bound workloads: off
    by default (RRAM_MC_GRAPH=1 turns it on).  Measured on MI355X / ROCm 7 it
    is slower than eager launches on every one of them, on torch's NULL stream
    (a private capture stream + 2 events per call) and on a created stream
    alike (profiles/r04_ab_graph.txt)."""
    return os.environ.get("RRAM_MC_GRAPH", "0") != "0"


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
        # 100 maps per step: the driver-style `--steps 10` runs BASELINE.json's
        # "1000 fault maps on one MI355X" in one line
        maps_per_step = 100
        mc = caffe.MonteCarlo(net, cfgs, seed=args.seed, max_maps=(args.steps + args.warmup) * maps_per_step + 8)
        mc.set_graph(_graph_on())         # replay each map as one hipGraph (opt-in, see _graph_on)
        el = _timed(world, dev, lambda i: mc.run((rank + world * i) * maps_per_step, maps_per_step),
                    args.steps, args.warmup)
        st = mc.stats()
        graph = mc.graph_active()
        # per-output mean / std / 95 % CI over the timed maps of every rank
        names = [k for k, v in net.outputs().items() if v.numel() == 1][:len(st["sums"])]
        rows = st["per_map"][args.warmup * maps_per_step:(args.warmup + args.steps) * maps_per_step]
        acc = []
        for k in range(len(names)):
            acc += [sum(r[k] for r in rows), sum(r[k] * r[k] for r in rows)]
        tot_m = allreduce_stats(acc + [len(rows)], dev)
        per_output = {name: map_statistics(tot_m[2 * k], tot_m[2 * k + 1], tot_m[-1]) for k, name in enumerate(names)}
        # the contraction table: events around every conv / IP layer over K
        # further maps after the timed region (the maps run eager while timed)
        net.layer_times(reset=True)
        net.set_timing(2)
        for i in range(args.steps):
            mc.run((rank + world * (args.warmup + args.steps + i)) * maps_per_step, maps_per_step)
        torch.cuda.synchronize()
        net.set_timing(0)
        tot = allreduce_stats(st["sums"] + [st["maps"]], dev)
        n_maps = world * args.steps * maps_per_step
        res = _base("Monte Carlo fault maps/sec, CIFAR-10 quick (quantised + lognormal)", "maps/s", n_maps / el,
                    world, args, el, workload="cifar10_quick_mc_quant16_lognormal0.1", model="CIFAR10_quick",
                    global_batch=batch * world, maps_per_step=maps_per_step * world, p_fault=0.01)
        res["images_per_s"] = round(n_maps * batch / el, 1)
        res["hipgraph"] = graph
        res["mc_mean_outputs"] = [x / max(tot[-1], 1) for x in tot[:-1]]
        res["mc_timed_maps"] = per_output     # mean, sample std and 95 % CI half-width over the timed maps
        res["roofline"] = contraction_roofline(net, args.steps * maps_per_step, net.layer_times())
        mc.close()
        net.close()
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cb = mc_cpu_baseline(models.cifar10_quick, "cifar10_quick", batch, cfgs, args.seed)
            cb.update(value=round(cb["value"] / batch, 4), unit="maps/s",
                      images_per_s=cb["value"])   # the metric is maps/s: one map = one `batch`-image pass
            res["cpu_baseline"] = cb
        return res

    if args.workload == "lenet_mc":
        batch = 100
        net = caffe.Net(models.lenet(test_batch=batch), "test", models.net_options("lenet"))
        mc = caffe.MonteCarlo(net, make_inject_cfg(args.p_fault), seed=args.seed,
                              max_maps=(args.steps + args.warmup) * 10 + 8)
        mc.set_graph(_graph_on())
        maps_per_step = 10
        el = _timed(world, dev, lambda i: mc.run((rank + world * i) * maps_per_step, maps_per_step),
                    args.steps, args.warmup)
        st = mc.stats()
        tot = allreduce_stats(st["sums"] + [st["maps"]], dev)
        n_img = world * args.steps * maps_per_step * batch
        res = _base("Monte Carlo fault-map inferences/sec, LeNet stuck-at", "images/s", n_img / el, world, args, el,
                    workload="lenet_mc_stuckat", model="LeNet (lenet_train_test TEST)", global_batch=batch * world,
                    maps_per_step=maps_per_step * world, p_fault=args.p_fault)
        res["mc_mean_outputs"] = [x / max(tot[-1], 1) for x in tot[:-1]]
        res["hipgraph"] = mc.graph_active()
        mc.close()
        net.close()
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = lenet_cpu_baseline(batch, args.p_fault, args.seed)
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
        opts = dict(opts, fused_update=True, conv_flip_cache=not getattr(args, "no_conv_flip_cache", False))
        # bucketed gradient all-reduce overlapped with backward (world > 1 only)
        dp = DataParallelSolver(sp, net_txt, opts, seed=args.seed, overlap=True)
        dp.solver.set_graph(_graph_on())  # iteration as two hipGraphs around the all-reduce (opt-in)
        # one Step call per region (the flipped kernels an update writes serve
        # the next backward within a call, Caffe::step_epoch)
        el = _timed(world, dev, None, args.steps, args.warmup, block=dp.step)
        res = _base(f"fault-aware training images/sec, {args.workload}", "images/s",
                    world * args.steps * batch / el, world, args, el, workload=args.workload,
                    model=args.workload.split("_")[0], global_batch=batch * world,
                    parallelism=f"dp{world} (RCCL all-reduce of {dp.num_params} fp32 grads"
                                f"{', bucketed, overlapped with backward' if dp.overlap else ''}; "
                                f"{'C++ host P2PSync (librram_caffe RCCL)' if dp.sync is not None else 'torch.distributed ' + dist.get_backend() if _dist_on() else 'no collective'})")
        res["broken_cells"] = sum(dp.solver.broken_counts())
        res["hipgraph"] = dp.solver.graph_active()
        # training roofline over the whole iteration: forward + weight-gradient +
        # data-gradient contractions (the first layer computes no data gradient;
        # the backward GEMMs run on the fp32 MFMA engine), against the step time
        con = dp.solver.net.contractions()
        fwd = sum(f for f, e in con.values())
        first = next(iter(con.values()))[0] if con else 0.0
        flops = 3 * fwd - first
        t_min = (sum(f / (PEAK_OF_ENGINE[e] * 1e12) for f, e in con.values())
                 + (2 * fwd - first) / (MFMA_F32_PEAK_TFLOPS * 1e12))
        ach = flops / (el / args.steps) / 1e12
        peak = flops / t_min / 1e12
        res["roofline"] = {"bound": "mfma", "achieved": round(ach, 3), "peak": round(peak, 1),
                           "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": None,
                           "algorithmic_flops_per_step": flops,
                           "kernel": "whole training iteration: forward (engine per layer) + backward dW / dX "
                                     "contractions (fp32 MFMA) of the Convolution / InnerProduct layers over the "
                                     "step time (includes the LRN / pool / loss / update / Fail kernels and the "
                                     "launch gaps of a batch-100 net)"}
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            # a CPU training iteration costs more than its TEST-phase forward:
            # the forward-only Caffe-CPU rate bounds the CPU training rate from above
            name = args.workload.split("_train")[0] if args.workload == "lenet_train" else "cifar10_full"
            fn = models.lenet if name == "lenet" else models.cifar10_full
            cb = mc_cpu_baseline(fn, name, batch, [make_inject_cfg(0.0)], args.seed, budget_s=5.0)
            cb["sample"] = ("UPPER BOUND on CPU training throughput: TEST-phase forward only, no backward / update. "
                            + cb["sample"])
            res["cpu_baseline"] = cb
        dp.close()
        return res

    if args.workload == "googlenet_sweep":
        batch = args.batch
        # RRAM_FUSE_CONCAT=0: the unfolded net (A/B of the TEST-phase Concat fold)
        fold = os.environ.get("RRAM_FUSE_CONCAT", "1") != "0"
        net = caffe.Net(models.googlenet(test_batch=batch), "test", models.net_options("googlenet", fuse_concat=fold))
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
        el = _timed(world, dev, step, args.steps, args.warmup, net)
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
        res["roofline"] = contraction_roofline(net, args.steps * len(rates), net.layer_times())
        for mc in mcs:
            mc.close()
        net.close()
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = mc_cpu_baseline(models.googlenet, "googlenet", batch, cfgs_for(0.01), args.seed)
        return res
    raise ValueError(args.workload)
