"""Kernel micro-benchmarks on the GPU (developer tool): injection / fail_apply
GB/s and conv / IP GEMM TFLOP/s at the AlexNet b256 shapes."""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))

import torch  # noqa: E402

from rramsim import make_inject_cfg, ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def micro(dev):
    """Practical ceilings: pure fp32-MFMA chains, a 16-B copy of the injection's
    bytes, and Philox4x32-10 calls/s without memory traffic (scripts/microbench.hip)."""
    import ctypes as C
    import subprocess
    so = ROOT / "scripts" / "_build" / "libmicro.so"
    src = ROOT / "scripts" / "microbench.hip"
    if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
        so.parent.mkdir(exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                               "-o", str(so), str(src)])
    lib = C.CDLL(str(so))
    st = lambda: C.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    out = {}
    o = torch.zeros(16, device=dev)
    blocks, iters = 256 * 8, 2000
    t = timeit(lambda: lib.micro_mfma_f32(C.c_void_p(o.data_ptr()), blocks, iters, st()), iters=5, warm=2)
    out["mfma_f32_peak_TFs"] = blocks * 4 * iters * 16 * 32 * 32 * 2 * 2 / t / 1e12
    t = timeit(lambda: lib.micro_mfma_f32_rand(C.c_void_p(o.data_ptr()), blocks, iters // 2, st()), iters=5, warm=2)
    out["mfma_f32_rand_TFs"] = blocks * 4 * (iters // 2) * 32 * 32 * 32 * 2 * 2 / t / 1e12
    t = timeit(lambda: lib.micro_lds_mfma(C.c_void_p(o.data_ptr()), 1024, 2000, st()), iters=5, warm=2)
    out["lds_mfma_core_TFs"] = 1024 * 2000 * 2.0 * 128 * 128 * 16 / t / 1e12
    n = 58_631_144 // 4 * 4
    x = torch.randn(n, device=dev)
    y = torch.empty_like(x)
    for nb in (2048, 8192, 32768):
        t = timeit(lambda: lib.micro_copy_f32(C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()),
                                              C.c_int64(n), nb, st()))
        out[f"copy16B_{nb}blk_GBps"] = 8 * n / t / 1e9
    u = torch.empty(256 * 8192, dtype=torch.int32, device=dev)
    cpt = 64
    t = timeit(lambda: lib.micro_philox(C.c_void_p(u.data_ptr()), 8192, C.c_int64(cpt), st()))
    out["philox_Gcalls_per_s"] = 256 * 8192 * cpt / t / 1e9
    out["philox_us_per_alexnet_map"] = 58_631_144 / 2 / (out["philox_Gcalls_per_s"] * 1e9) * 1e6
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    res = {}
    if a.only in ("", "inject"):
        shapes = [(4096, 9216), (4096,), (4096, 4096), (4096,), (1000, 4096), (1000,)]
        c = make_inject_cfg(0.01)
        srcs = [torch.randn(s, device=dev) for s in shapes]
        outs = [torch.empty_like(x) for x in srcs]
        segs = [(s, o, i, c) for i, (s, o) in enumerate(zip(srcs, outs))]
        n = sum(x.numel() for x in srcs)
        m = [0]

        def run():
            m[0] += 1
            ops.inject_batched(segs, 1701, m[0])
        t = timeit(run)
        res["inject_GBps"] = 8 * n / t / 1e9
        res["inject_us"] = t * 1e6
        dw = [torch.randn_like(x) for x in srcs]
        e = [torch.full_like(x, 1e6) for x in srcs]
        v = [torch.zeros_like(x) for x in srcs]
        fsegs = list(zip(dw, outs, e, v))
        t = timeit(lambda: ops.fail_apply_batched(fsegs))
        res["fail_apply_GBps"] = 16 * n / t / 1e9   # e R/W, v R, dw R (w not written)
        res["fail_apply_us"] = t * 1e6
        x = torch.randn(n, device=dev)
        y = torch.empty_like(x)
        t = timeit(lambda: y.copy_(x))
        res["copy_GBps"] = 8 * n / t / 1e9
    if a.only == "dense":
        # the conv layers' GEMM shapes with dense operands (C = A B^T, float4 loads on
        # both sides): what the same MFMA core reaches without the implicit-im2col gather
        for name, M, N, K in (("dense_conv3", 384, 43264, 2304), ("dense_conv2g", 128, 186624, 1200),
                              ("dense_conv1", 96, 774400, 364), ("dense_4096", 4096, 4096, 4096)):
            A = torch.randn(M, K, device=dev) * 0.01
            Bm = torch.randn(N, K, device=dev)
            Cm = torch.empty(M, N, device=dev)
            t = timeit(lambda: ops.gemm(0, 1, M, N, K, 1.0, A, Bm, 0.0, Cm), iters=5)
            res[f"{name}_TFs"] = 2.0 * M * N * K / t / 1e12
            res[f"{name}_ms"] = t * 1e3
    if a.only == "vendor":
        # the vendor libraries on the same box, for reference only (never on the product
        # path): torch.mm = hipBLASLt / rocBLAS sgemm, F.conv2d = MIOpen, all fp32
        torch.backends.cuda.matmul.allow_tf32 = False
        torch.backends.cudnn.allow_tf32 = False
        for name, M, N, K in (("sq4096", 4096, 4096, 4096), ("dense_conv3", 384, 43264, 2304),
                              ("dense_conv2g", 128, 186624, 1200), ("fc6", 256, 4096, 9216),
                              ("fc7", 256, 4096, 4096), ("fc8", 256, 1000, 4096)):
            A = torch.randn(M, K, device=dev)
            Bm = torch.randn(N, K, device=dev)
            t = timeit(lambda: torch.mm(A, Bm.t()), iters=5)
            res[f"vendor_mm_{name}_TFs"] = 2.0 * M * N * K / t / 1e12
        import torch.nn.functional as F
        B = 256
        tot_f = tot_t = 0.0
        for name, xs, co, k, s, p, g in (("conv1", (B, 3, 227, 227), 96, 11, 4, 0, 1),
                                         ("conv2", (B, 96, 27, 27), 256, 5, 1, 2, 2),
                                         ("conv3", (B, 256, 13, 13), 384, 3, 1, 1, 1),
                                         ("conv4", (B, 384, 13, 13), 384, 3, 1, 1, 2),
                                         ("conv5", (B, 384, 13, 13), 256, 3, 1, 1, 2)):
            x = torch.randn(xs, device=dev)
            w = torch.randn(co, xs[1] // g, k, k, device=dev) * 0.01
            b = torch.randn(co, device=dev)
            y = F.conv2d(x, w, b, stride=s, padding=p, groups=g)
            t = timeit(lambda: F.conv2d(x, w, b, stride=s, padding=p, groups=g), iters=5)
            fl = 2.0 * B * co * y.shape[2] * y.shape[3] * (xs[1] // g) * k * k
            res[f"vendor_conv_{name}_TFs"] = fl / t / 1e12
            res[f"vendor_conv_{name}_ms"] = t * 1e3
            tot_f += fl
            tot_t += t
        res["vendor_conv_total_ms"] = tot_t * 1e3
        res["vendor_conv_TFs"] = tot_f / tot_t / 1e12
    if a.only in ("", "gemm"):
        B = 256
        convs = [("conv1", (B, 3, 227, 227), 96, 11, 4, 0, 1), ("conv2", (B, 96, 27, 27), 256, 5, 1, 2, 2),
                 ("conv3", (B, 256, 13, 13), 384, 3, 1, 1, 1), ("conv4", (B, 384, 13, 13), 384, 3, 1, 1, 2),
                 ("conv5", (B, 384, 13, 13), 256, 3, 1, 1, 2)]
        tot_f, tot_t = 0.0, 0.0
        for name, xs, co, k, s, p, g in convs:
            d = ops.conv_desc(xs, co, k, s, p, 1, g)
            x = torch.randn(xs, device=dev)
            w = torch.randn(co, xs[1] // g, k, k, device=dev) * 0.01
            b = torch.randn(co, device=dev)
            y = torch.empty(B, co, d.out_h, d.out_w, device=dev)
            t = timeit(lambda: ops.conv2d_fwd(d, x, w, b, y, True), iters=5)
            fl = 2.0 * B * co * d.out_h * d.out_w * (xs[1] // g) * k * k
            res[f"{name}_TFs"] = fl / t / 1e12
            res[f"{name}_ms"] = t * 1e3
            tot_f += fl
            tot_t += t
        ws = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
        for name, M, N, K in (("fc6", B, 4096, 9216), ("fc7", B, 4096, 4096), ("fc8", B, 1000, 4096)):
            X = torch.randn(M, K, device=dev)
            W = torch.randn(N, K, device=dev) * 0.01
            bb = torch.randn(N, device=dev)
            Y = torch.empty(M, N, device=dev)
            t = timeit(lambda: ops.ip_fwd(X, W, bb, Y, M, N, K, relu=True, workspace=ws), iters=10)
            fl = 2.0 * M * N * K
            res[f"{name}_TFs"] = fl / t / 1e12
            res[f"{name}_ms"] = t * 1e3
            tot_f += fl
            tot_t += t
        res["alexnet_gemm_TFs"] = tot_f / tot_t / 1e12
        res["alexnet_gemm_ms"] = tot_t * 1e3
        M = N = K = 4096
        A = torch.randn(M, K, device=dev)
        Bm = torch.randn(K, N, device=dev)
        Cm = torch.empty(M, N, device=dev)
        t = timeit(lambda: ops.gemm(0, 0, M, N, K, 1.0, A, Bm, 0.0, Cm), iters=5)
        res["sq4096_TFs"] = 2.0 * M * N * K / t / 1e12
    if a.only in ("", "micro"):
        res.update(micro(dev))
    for k, v in res.items():
        print(f"{k:>20s} {v:10.3f}")


if __name__ == "__main__":
    main()
