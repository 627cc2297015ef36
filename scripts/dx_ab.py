"""Developer A/B: conv data-gradient time (rram_conv2d_bwd with dX only) per
shape, for RRAM_DX_FWD=0 (data GEMM + col2im) vs 1 (flipped-kernel forward).
Run once per setting; prints one JSON line per shape."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))
import torch  # noqa: E402

from rramsim import ops  # noqa: E402

SHAPES = [  # name, (n, c, h, w), cout, k, pad, group
    ("cifar_conv2", (100, 32, 16, 16), 32, 5, 2, 1),
    ("cifar_conv3", (100, 32, 8, 8), 64, 5, 2, 1),
    ("lenet_conv2", (64, 20, 12, 12), 50, 5, 0, 1),
    ("alex_conv2", (64, 96, 27, 27), 256, 5, 2, 2),
    ("alex_conv3", (64, 256, 13, 13), 384, 3, 1, 1),
    ("alex_conv4", (64, 384, 13, 13), 384, 3, 1, 2),
    ("alex_conv5", (64, 384, 13, 13), 256, 3, 1, 2),
    ("gn_3x3", (32, 96, 28, 28), 128, 3, 1, 1),
    ("gn_1x1", (32, 256, 28, 28), 64, 1, 0, 1),
]


def main():
    dev = torch.device("cuda:0")
    mode = os.environ.get("RRAM_DX_FWD", "1")
    for eng_name, eng in (("f32", ops.ENGINE_F32), ("bf16x6", ops.ENGINE_BF16X6)):
        prev = ops.set_f32_engine(eng)
        for name, xs, cout, k, p, g in SHAPES:
            d = ops.conv_desc(xs, cout, k, 1, p, 1, g)
            x = torch.randn(xs, device=dev)
            w = torch.randn(cout, xs[1] // g, k, k, device=dev) * 0.1
            dy = torch.randn(xs[0], cout, d.out_h, d.out_w, device=dev)
            dx = torch.empty_like(x)
            ws = torch.empty(ops.conv2d_bwd_workspace(d, xs[0]) // 4 + 64, device=dev)
            fn = lambda: ops.conv2d_bwd(d, x, w, dy, None, None, dx, ws)  # noqa: E731
            for _ in range(3):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(20):
                fn()
            e.record()
            torch.cuda.synchronize()
            print(json.dumps({"dx_fwd": mode, "engine": eng_name, "shape": name, "us": round(s.elapsed_time(e) / 20 * 1e3, 1)}),
                  flush=True)
        ops.set_f32_engine(prev)


if __name__ == "__main__":
    main()
