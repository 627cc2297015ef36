#!/usr/bin/env python3
"""Headline benchmark: Monte-Carlo fault-map inference, AlexNet b256.

One step = one fault map on every rank: inject a fresh stuck-at fault map into
the clean InnerProduct weights (counter-based RNG, HBM-bound kernel), then run
the full AlexNet forward over the 256-image eval batch (implicit-GEMM conv and
IP GEMMs with fp32 products on the matrix cores — fp32 MFMA, or the exact
bf16x6 split for the 3x3 / 5x5 convolutions and fc6/fc7 —,
LRN/pool/softmax/accuracy), accumulating accuracy and
loss on the device.  Maps are sharded across ranks (map m on rank m mod N; no
data-path collective); one RCCL all-reduce of the statistics closes the job.

Prints ONE JSON line (rank 0):
  value = images classified under faults per second, summed over ranks
  roofline = the dominant kernel (conv2, k_conv_cb16_x6 5x5) vs the peak of
             its engine (bf16x6 split: bf16 dense peak / 6), hipEvents around
             its layer in the timed region; `contractions` = all conv / IP
             layers vs their engines' peaks, timed over K further maps after
             the timed region (events around 8 layers cost ~1 % of a step)
  roofline_inject = the injection kernel vs HBM peak
  cpu_baseline = Caffe CPU mode restated in C (oracle/caffe_cpu.c: per-image
                 im2col + cblas_sgemm, Fail_cpu) over one full map, rank 0 at N=1.

Launch: python bench.py [--gpus N --steps K --warmup W]
        torchrun --nproc-per-node N bench.py --gpus N ...  (one rank per GPU, RCCL)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))

MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: fp32 MFMA = fp32 vector peak (dense)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: bf16 dense MFMA (no sparsity)
# the bf16x6 engine (include/rram_kernels.h) spends 6 bf16 MFMA products per
# fp32 product: its roofline is the bf16 dense peak / 6 in fp32 FLOPs
MFMA_X6_PEAK_TFLOPS = MFMA_BF16_PEAK_TFLOPS / 6.0
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
# the dominant kernel of the step: conv2's k_conv_cb16_x6<5,5,4,4,8,2,1> (23 %
# of GPU time, profiles/r06f_bench_kernel_stats.csv); the only layer timed
# inside the timed region, so the stream carries two markers per map for it
DOMINANT_LAYER = "conv2"
DOMINANT_PMC_CLASS = "conv2 k_conv_cb16_x6<5,5,...>"


def alexnet_gemm_table(batch):
    """(layer, FLOPs per batch) for AlexNet at 227x227."""
    convs = [("conv1", 96, 3, 11, 55, 1), ("conv2", 256, 96, 5, 27, 2), ("conv3", 384, 256, 3, 13, 1),
             ("conv4", 384, 384, 3, 13, 2), ("conv5", 256, 384, 3, 13, 2)]
    t = {}
    for name, co, ci, k, o, g in convs:
        t[name] = 2.0 * batch * co * o * o * (ci // g) * k * k
    for name, n, k in (("fc6", 4096, 9216), ("fc7", 4096, 4096), ("fc8", 1000, 4096)):
        t[name] = 2.0 * batch * n * k
    return t


def alexnet_engines(batch):
    """Engine each AlexNet conv / IP layer runs on (rram_f32_engine_for_*)."""
    from rramsim import ops
    convs = {"conv1": ((batch, 3, 227, 227), 96, 11, 4, 0, 1), "conv2": ((batch, 96, 27, 27), 256, 5, 1, 2, 2),
             "conv3": ((batch, 256, 13, 13), 384, 3, 1, 1, 1), "conv4": ((batch, 384, 13, 13), 384, 3, 1, 1, 2),
             "conv5": ((batch, 384, 13, 13), 256, 3, 1, 1, 2)}
    eng = {}
    for name, (x, co, k, st, pd, g) in convs.items():
        eng[name] = ops.f32_engine_for_conv(ops.conv_desc(x, co, k, st, pd, 1, g))
    for name, n, k in (("fc6", 4096, 9216), ("fc7", 4096, 4096), ("fc8", 1000, 4096)):
        eng[name] = ops.f32_engine_for_ip(batch, n, k)
    return {k: ("bf16x6" if v == ops.ENGINE_BF16X6 else "f32") for k, v in eng.items()}


def cpu_baseline(batch, p_fault, seed):
    """Caffe CPU mode restated in C (oracle/caffe_cpu.c): one
    full Monte-Carlo map of AlexNet b`batch` on this host's physical cores
    (affinity set / SMT) — the GaussianFailureMaker draws + Fail_cpu over the
    58,631,144 IP cells, then the TEST forward of all `batch` images in the
    reference's layer order (per-image im2col_cpu + cblas_sgemm per group,
    single-threaded LRN / pool / ReLU loops).  Not extrapolated: the whole map
    is timed.  The same map also runs with sgemm on the box's per-GPU CPU
    share (OMP_NUM_THREADS); the faster of the two is the baseline and both
    are reported (`by_threads`)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    phys = oracle.physical_cores()
    env = os.environ.get("OMP_NUM_THREADS", "")
    share = int(env) if env.isdigit() else 0
    runs = []
    for th in sorted({phys} | ({share} if 0 < share < phys else set())):
        t, meta = oracle.caffe_cpu_alexnet_map(batch=batch, p_fault=p_fault, seed=seed, threads=th)
        runs.append((batch / sum(t.values()), th, t, meta))
    # the faster thread count is the baseline (OpenBLAS over all physical cores
    # of a shared box can lose to the per-GPU share on per-image GEMMs)
    best = max(runs, key=lambda r: r[0])
    v, th, t, meta = best
    res = {"value": round(v, 3), "unit": "images/s", "cores": th, "kind": "port",
           "sample": f"1 full fault map: {meta['broken_cells']} of 58,631,144 IP cells broken + {batch}-image "
                     f"AlexNet TEST forward, {sum(t.values()):.2f} s; sgemm = {meta['blas']} on {th} threads, other "
                     f"layers single-threaded as in Caffe; host: {meta['affinity_cpus']} CPUs in the affinity set = "
                     f"{phys} physical cores, OMP_NUM_THREADS {env or 'unset'}",
           "layers_ms": {k: round(x * 1e3, 1) for k, x in t.items()},
           "by_threads": {str(r[1]): round(r[0], 3) for r in runs}}
    return res


def load_traffic():
    """HBM bytes from the committed rocprofv3 PMC passes of this same command
    (scripts/pmc.sh + scripts/pmc_traffic.py -> profiles/pmc_traffic.json):
    PMC counters cannot be read from inside the timed process itself."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    try:
        return json.loads(p.read_text())
    except (OSError, ValueError):
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--p-fault", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=1701)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-layers", action="store_true", help="print the per-layer table to stderr")
    ap.add_argument("--no-conv-flip-cache", action="store_true",
                    help="training workloads: flip each convolution kernel per backward instead of taking the copy "
                         "the fused update wrote (net option conv_flip_cache; A/B runs)")
    ap.add_argument("--layer-events", choices=["dominant", "none"], default="dominant",
                    help="hipEvents in the timed region: around the dominant kernel's layer (roofline) or none")
    ap.add_argument("--workload", default="alexnet_mc",
                    choices=["alexnet_mc", "alexnet_mc_reuse_prefix", "cifar10_quick_mc", "cifar10_full_train",
                             "googlenet_sweep", "lenet_train", "lenet_mc"],
                    help="alexnet_mc is the headline (BASELINE.json metric); alexnet_mc_reuse_prefix runs the "
                         "fault-free conv1..pool5 prefix once (MonteCarlo prefix reuse: a different workload, never "
                         "the headline); the others are the remaining configs")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from rramsim import caffe, make_inject_cfg, models

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; RRAM_BENCH_DIST_BACKEND=gloo (test hook) lets a box with
    # fewer GPUs than ranks rehearse the N > 1 path, ranks then share devices
    backend = os.environ.get("RRAM_BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # under torch.distributed.run the process group exists at every world
    # size (N = 1 included), so the collectives below are the ones N > 1 runs
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    comm = None
    if distributed:
        # torch.distributed is the rendezvous only (gloo over TCP on the host):
        # with RCCL (the default) every collective of the job -- the timing
        # barriers, the max-over-ranks time, the statistics and the training
        # gradients -- runs on the C++ host's own RCCL communicator
        # (caffe.Comm / P2PSync, host/parallel.cpp); RRAM_BENCH_DIST_BACKEND=gloo
        # (test hook, ranks sharing one GPU) keeps them on torch's gloo
        dist.init_process_group("gloo")
        if backend == "nccl":
            from rramsim import parallel
            comm = caffe.Comm(rank, world)
            parallel.set_comm(comm)
    if os.environ.get("RRAM_BENCH_STREAM") == "1":   # A/B runs: a created stream instead of the NULL stream
        torch.cuda.set_stream(torch.cuda.Stream())
    caffe.set_stream_from_torch()
    caffe.set_random_seed(args.seed)
    if args.workload not in ("alexnet_mc", "alexnet_mc_reuse_prefix"):
        sys.path.insert(0, str(ROOT / "scripts"))
        from bench_workloads import run_workload
        res = run_workload(args, world, rank, dev)
        if rank == 0:
            print(json.dumps(res), flush=True)
        _finish(comm, distributed)
        return

    net = caffe.Net(models.alexnet(test_batch=args.batch), "test", models.net_options("alexnet"))
    cfg = make_inject_cfg(args.p_fault)             # reference stuck-at semantics, neg/zero/pos 10/20/10
    mc = caffe.MonteCarlo(net, cfg, seed=args.seed, max_maps=2 * args.steps + args.warmup + 8)
    reuse = args.workload == "alexnet_mc_reuse_prefix"
    if reuse:
        mc.set_reuse_prefix(True)   # conv1..pool5 once (fixed batch, IP-only faults); each map: inject + fc6..
    dom_layer = "fc6" if reuse else DOMINANT_LAYER

    def step(i):
        mc.run(rank + world * i, 1)                 # map m on rank m mod N

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    mc.reset()
    net.layer_times(reset=True)
    mc.inject_times(reset=True)
    if args.profile_layers:
        net.set_timing(1)
    elif args.layer_events == "dominant":
        net.set_timing_layer(dom_layer)
    else:
        net.set_timing(0)
    mc.set_timing(True)

    stats = torch.zeros(8, dtype=torch.float64)
    if comm is not None:
        comm.barrier()
    elif distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    net.set_timing(False)
    mc.set_timing(False)
    st = mc.stats()
    if comm is not None:
        # one RCCL all-reduce of [output sums, broken cells, maps] from the C++ host
        vals = comm.mc_stats(mc)
        elapsed = comm.allreduce_host([elapsed], "max")[0]
        comm.barrier()
    else:
        vals = st["sums"] + [float(sum(st["broken"])), float(st["maps"])]
        if distributed:
            t = torch.tensor(vals + [elapsed], dtype=torch.float64)
            dist.all_reduce(t[:len(vals)])             # gloo rehearsal: accuracy / loss / broken-cell sums
            dist.all_reduce(t[len(vals):], op=dist.ReduceOp.MAX)
            dist.barrier()
            vals, elapsed = t[:len(vals)].tolist(), float(t[-1].item())
    stats[:len(vals)] = torch.tensor(vals, dtype=torch.float64)
    torch.cuda.synchronize()

    # ---- roofline of the dominant kernel: live hipEvents of the timed region
    lt_timed = net.layer_times(reset=True)
    # ---- contraction table: K further maps, untimed for `value`, with events
    # around every conv / IP layer (each rank on its own maps, no collective)
    if not args.profile_layers:
        net.set_timing(2)
        for i in range(args.steps):
            step(args.warmup + args.steps + i)
        torch.cuda.synchronize()
        net.set_timing(False)
        lt = net.layer_times()
    else:
        lt = lt_timed
    flops = alexnet_gemm_table(args.batch)
    engines = alexnet_engines(args.batch)
    ran = {name for (name, typ, ms, cnt) in lt if name in flops and cnt > 0}   # prefix reuse: fc6-8 only
    flops = {n: f for n, f in flops.items() if n in ran}
    gemm_ms = sum(ms for (name, typ, ms, cnt) in lt if name in flops) / args.steps
    gemm_flops = sum(flops.values())
    achieved_tf = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else 0.0
    # the roofline of the mixed-engine layer set: each layer's FLOPs at its
    # engine's peak; effective peak = total FLOPs / that minimum time
    peak_of = {"f32": MFMA_F32_PEAK_TFLOPS, "bf16x6": MFMA_X6_PEAK_TFLOPS}
    t_min = sum(f / (peak_of[engines[n]] * 1e12) for n, f in flops.items())
    peak_tf = gemm_flops / t_min / 1e12
    layers = {name: {"engine": engines[name], "ms": round(ms / args.steps, 4),
                     "tflops": round(flops[name] / (ms / args.steps * 1e-3) / 1e12, 1) if ms > 0 else None}
              for (name, typ, ms, cnt) in lt if name in flops}
    inj_ms, inj_n, inj_w = mc.inject_times()
    inj_ms_per = inj_ms / max(inj_n, 1)
    inj_gbps = 8.0 * inj_w / (inj_ms_per * 1e-3) / 1e9
    if args.profile_layers and rank == 0:
        for name, typ, ms, cnt in lt:
            print(f"{name:>12s} {typ:>16s} {ms / max(cnt, 1):9.3f} ms", file=sys.stderr)

    traffic = load_traffic()
    dom_ms = {name: ms for (name, typ, ms, cnt) in lt_timed}.get(dom_layer, 0.0) / args.steps
    dom_flops = alexnet_gemm_table(args.batch)[dom_layer]
    dom_tf = dom_flops / (dom_ms * 1e-3) / 1e12 if dom_ms > 0 else 0.0
    dom_peak = peak_of[engines[dom_layer]]
    dom_pmc = {} if reuse else traffic.get("per_kernel", {}).get(DOMINANT_PMC_CLASS, {})
    n_images = world * args.steps * args.batch
    value = n_images / elapsed
    out_names = [k for k in net.outputs().keys()]
    mean_out = {nm: float(stats[k].item()) / max(1.0, float(stats[len(st["sums"]) + 1].item()))
                for k, nm in enumerate(out_names[:len(st["sums"])])}
    res = {
        "metric": "Monte Carlo fault-map inferences/sec, AlexNet b256" + (
            ", fault-free prefix reused (not the reference workload)" if reuse else ""),
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (bf16x6 products)" if "bf16x6" in engines.values() else "f32",
        "data": "synthetic (U{0..255}-128 images 3x227x227, random labels; seeded Caffe-filler weights)",
        "config": {"workload": "alexnet_b256_mc_faultmap_inference" + ("_prefix_reused" if reuse else ""),
                   "model": "AlexNet (bvlc_alexnet train_val, TEST)",
                   "global_batch": args.batch * world, "batch_per_map": args.batch, "maps_per_step": world,
                   "p_fault": args.p_fault, "stuck_split_neg_zero_pos": [10, 20, 10],
                   "fault_layers": "InnerProduct (58,631,144 weights)",
                   "parallelism": (f"mc-maps x{world} (RCCL stats all-reduce from the C++ host, rram_mc_allreduce_stats)"
                                   if comm is not None else f"mc-maps x{world} (torch {backend} stats all-reduce)"
                                   if distributed else "mc-maps x1 (single process, no collective)"),
                   "f32_engine": "bf16x6 (exact 3-term bf16 split, 6 products, fp32 accumulation)"
                   if "bf16x6" in engines.values() else "f32 MFMA"},
        "roofline": {"bound": "mfma", "achieved": round(dom_tf, 2), "peak": round(dom_peak, 1), "unit": "TFLOP/s",
                     "frac": round(dom_tf / dom_peak, 4),
                     "traffic": (dom_pmc["measured_MB_per_step"] * 1e6 if dom_pmc.get("measured_MB_per_step")
                                 else None),
                     "kernel": ("k_gemm_x6 (fc6, the largest per-map contraction with the prefix reused) "
                                if reuse else "k_conv_cb16_x6<5,5,4,4,8,2,1> (5x5 channel-octet kernel on "
                                "v_mfma_f32_16x16x32_bf16, 128 x 128 per-image tiles, two workgroups per CU)")
                               + f" = AlexNet {dom_layer} ({engines[dom_layer]} engine, "
                               "one launch per map), hipEvents around its layer over the timed region; peak = "
                               "bf16 dense 2500 / 6 products = 416.7 (f32 engine: v_mfma_f32_32x32x2_f32 157.3)",
                     "algorithmic_flops_per_launch": dom_flops,
                     "algorithmic_bytes_per_launch": (dom_pmc["algorithmic_MB_per_step"] * 1e6
                                                      if dom_pmc.get("algorithmic_MB_per_step") else None),
                     "avg_us_per_launch": round(dom_ms * 1e3, 2),
                     "contractions": {
                         "achieved": round(achieved_tf, 2), "peak": round(peak_tf, 1), "unit": "TFLOP/s",
                         "frac": round(achieved_tf / peak_tf, 4) if peak_tf else None,
                         "frac_of_f32_mfma_peak": round(achieved_tf / MFMA_F32_PEAK_TFLOPS, 4),
                         "traffic": traffic.get("gemm", {}).get("bytes_per_step"),
                         "algorithmic_flops_per_step": gemm_flops, "avg_ms_per_step": round(gemm_ms, 4),
                         "layers": layers,
                         "note": ("conv1-5 + fc6-8 forward, each layer at its engine's peak; hipEvents around every "
                                  "conv / IP layer over K further maps after the timed region"
                                  if not args.profile_layers else "every layer timed inside the timed region")}},
        "roofline_inject": {"bound": "hbm", "achieved": round(inj_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                            "frac": round(inj_gbps / HBM_PEAK_GBPS, 4),
                            "traffic": traffic.get("inject", {}).get("bytes_per_launch"),
                            "algorithmic_bytes_per_launch": 8 * inj_w, "avg_us_per_launch": round(inj_ms_per * 1e3, 2),
                            "note": ("launched on a side stream after conv2, overlapped with norm2 / pool2 / "
                                     "conv3-5 of the same map (RRAM_MC_OVERLAP=1; they share the CUs, so the "
                                     "launch stretches)"
                                     if os.environ.get("RRAM_MC_OVERLAP", "0") == "1" else
                                     "serial: each map's injection runs alone before its forward")},
        "traffic_source": traffic.get("source"),
        "mc_stats": {"maps": int(stats[len(st["sums"]) + 1].item()), "mean_outputs": mean_out,
                     "broken_cells": int(stats[len(st["sums"])].item())},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.batch, args.p_fault, args.seed)
    elif rank == 0:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    mc.close()
    net.close()
    _finish(comm, distributed)


def _finish(comm, distributed):
    import torch.distributed as dist
    if comm is not None:
        from rramsim import parallel
        parallel.set_comm(None)
        comm.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
