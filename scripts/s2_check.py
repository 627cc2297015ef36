"""GoogLeNet conv1 (b256, 3x224x224 -> 64x112x112, 7x7 / 2, pad 3) on the
bf16x6 engine (k_conv_s2_x6): kernel time and TFLOP/s against the 416.7 roof.
Developer tool: `python scripts/s2_check.py [--batch N] [--iters K]`."""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))

import torch  # noqa: E402

from rramsim import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(a.batch, 3, 224, 224, generator=g, device=dev)
    w = torch.randn(64, 3, 7, 7, generator=g, device=dev) * 0.05
    b = torch.randn(64, generator=g, device=dev) * 0.1
    d = ops.conv_desc(tuple(x.shape), 64, 7, 2, 3, 1, 1)
    y = torch.empty(a.batch, 64, 112, 112, device=dev)
    for _ in range(3):
        ops.conv2d_fwd(d, x, w, b, y, relu=True)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(a.iters):
        ops.conv2d_fwd(d, x, w, b, y, relu=True)
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / a.iters * 1e-3
    fl = 2.0 * a.batch * 64 * 147 * 112 * 112
    print(json.dumps({"engine": ops.f32_engine_for_conv(d), "us": round(t * 1e6, 1), "tflops": round(fl / t / 1e12, 1),
                      "frac_416.7": round(fl / t / 1e12 / 416.7, 3)}))


if __name__ == "__main__":
    main()
