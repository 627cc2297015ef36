"""AlexNet conv1 (b256, 3x227x227 -> 96x55x55) on the bf16x6 engine: error
against a float64 evaluation (as a fraction of sum |a*b|) and kernel time.
Developer tool: `python scripts/conv1_check.py [--batch N]`."""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from rramsim import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    x = (torch.randint(0, 256, (a.batch, 3, 227, 227), generator=g, device=dev).float() - 128.0)
    w = torch.randn(96, 3, 11, 11, generator=g, device=dev) * 0.01
    b = torch.randn(96, generator=g, device=dev) * 0.1
    d = ops.conv_desc(tuple(x.shape), 96, 11, 4, 0, 1, 1)
    y = torch.empty(a.batch, 96, 55, 55, device=dev)
    res = {"engine": ops.f32_engine_for_conv(d)}
    ops.conv2d_fwd(d, x, w, b, y, relu=False)
    torch.cuda.synchronize()
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=4)
    mag = F.conv2d(x.double().abs(), w.double().abs(), b.double().abs(), stride=4)
    err = ((y.double() - ref).abs() / mag.clamp_min(1e-30)).max().item()
    res["max_err_frac_sum_abs"] = err
    # where it goes wrong: per image and per 256-position tile of an image
    rel = ((y.double() - ref).abs() / mag.clamp_min(1e-30)).amax(dim=1).reshape(a.batch, -1)
    bad_img = (rel.amax(dim=1) > 1e-4).nonzero().flatten().tolist()
    res["bad_images"] = bad_img[:20] + (["..."] if len(bad_img) > 20 else [])
    if bad_img:
        i0 = bad_img[0]
        tiles = [float(rel[i0, k * 256:(k + 1) * 256].max()) for k in range((rel.shape[1] + 255) // 256)]
        res["first_bad_image_tile_err"] = [round(t, 4) for t in tiles]
        res["bad_channels"] = ((y.double() - ref).abs() / mag.clamp_min(1e-30))[i0].reshape(96, -1).amax(dim=1).gt(1e-4).nonzero().flatten().tolist()[:20]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        ops.conv2d_fwd(d, x, w, b, y)
    torch.cuda.synchronize()
    s.record()
    for _ in range(a.iters):
        ops.conv2d_fwd(d, x, w, b, y)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    flops = 2.0 * a.batch * 96 * 55 * 55 * 363
    res.update(ms=round(ms, 4), tflops=round(flops / ms / 1e9, 1))
    print(json.dumps(res))
    if err >= 1e-4:
        sys.exit(1)


if __name__ == "__main__":
    main()
