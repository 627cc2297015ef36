"""Developer probe: bf16x6 vs fp32-MFMA engine on extreme operand ranges
(conv: channel-octet / conv1 / patch kernels; IP: k_gemm_x6), against a
float64 evaluation (error / sum|a*b|) and the NaN / +-Inf pattern of a CPU
float32 evaluation.  `python scripts/x6_range_probe.py`"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from rramsim import ops  # noqa: E402

dev = torch.device("cuda", 0)
CONVS = {"cb3x3": ((2, 256, 13, 13), 384, 3, 1, 1), "conv1": ((2, 3, 227, 227), 96, 11, 4, 0),
         "patch": ((2, 24, 20, 20), 96, 3, 1, 1)}


def run_conv(name, x, w, eng):
    xs, co, k, s, p = CONVS[name]
    d = ops.conv_desc(xs, co, k, s, p, 1, 1)
    prev = ops.set_f32_engine(eng)
    y = torch.empty(xs[0], co, d.out_h, d.out_w, device=dev)
    ops.conv2d_fwd(d, x.to(dev), w.to(dev), None, y)
    ops.set_f32_engine(prev)
    torch.cuda.synchronize()
    ref = F.conv2d(x.double(), w.double(), stride=s, padding=p)
    mag = F.conv2d(x.double().abs(), w.double().abs(), stride=s, padding=p)
    r32 = F.conv2d(x, w, stride=s, padding=p)
    return y.cpu(), ref, mag, r32


def run_ip(x, w, eng):
    M, K = x.shape
    N = w.shape[0]
    prev = ops.set_f32_engine(eng)
    y = torch.empty(M, N, device=dev)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    ops.ip_fwd(x.to(dev), w.to(dev), None, y, M, N, K, workspace=ws)
    ops.set_f32_engine(prev)
    torch.cuda.synchronize()
    return y.cpu(), x.double() @ w.double().T, x.double().abs() @ w.double().abs().T, x @ w.T


def summary(got, ref, mag, r32):
    fin = torch.isfinite(r32) & torch.isfinite(ref)
    e = ((got.double() - ref).abs() / mag.clamp_min(1e-300))[fin & torch.isfinite(got)]
    return {"max_err_frac": float(e.max()) if e.numel() else None,
            "nan_match": bool(torch.equal(torch.isnan(got), torch.isnan(r32))),
            "posinf_match": bool(torch.equal(torch.isposinf(got), torch.isposinf(r32))),
            "neginf_match": bool(torch.equal(torch.isneginf(got), torch.isneginf(r32))),
            "n_nan": int(torch.isnan(got).sum()), "n_nan_ref": int(torch.isnan(r32).sum()),
            "n_inf": int(torch.isinf(got).sum()), "n_inf_ref": int(torch.isinf(r32).sum()),
            "finite_ok": bool(torch.isfinite(got)[fin].all())}


def cases(shape_x, shape_w, g):
    x = torch.randn(*shape_x, generator=g)
    w = torch.randn(*shape_w, generator=g) * 0.05
    out = {}
    xi = x.clone()
    xi.view(-1)[::997] = float("inf")
    xi.view(-1)[5::1993] = -float("inf")
    out["inf_inputs"] = (xi, w)
    wz = w.clone()
    wz.view(-1)[::7] = 0.0
    out["inf_inputs_zero_weights"] = (xi, wz)
    out["near_flt_max"] = (x * 3.0e37 / x.abs().max(), w / w.abs().max())
    out["above_bf16_max"] = (torch.where(x > 2.0, torch.full_like(x, 3.401e38), x), w * 1e-3)
    out["tiny_2m100"] = (x * 2.0 ** -100, w)
    out["tiny_2m115"] = (x * 2.0 ** -115, w * 2.0 ** 60)
    out["tiny_2m124"] = (x * 2.0 ** -124, w * 2.0 ** 60)
    out["denormal_inputs"] = (x * 2.0 ** -135, w * 2.0 ** 100)
    out["big_x_tiny_w"] = (x * 2.0 ** 60, w * 2.0 ** -120)
    return out


res = {}
g = torch.Generator().manual_seed(3)
for name, (xs, co, k, s, p) in CONVS.items():
    for cname, (x, w) in cases(xs, (co, xs[1], k, k), g).items():
        for eng in (1, 0):
            res[f"conv {name} {cname} eng{eng}"] = summary(*run_conv(name, x, w, eng))
for cname, (x, w) in cases((256, 9216), (4096, 9216), g).items():
    for eng in (1, 0):
        res[f"ip fc6 {cname} eng{eng}"] = summary(*run_ip(x, w, eng))
for k, v in res.items():
    print(k, json.dumps(v))
