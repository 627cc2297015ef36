import sys, numpy as np, torch
sys.path.insert(0, "rram-caffe-simulation_amd/python"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
from rramsim import ops
import importlib
dev = torch.device("cuda", 0)
for (xs, co, k, g) in [((2, 1, 12, 12), 20, 5, 1), ((2, 3, 9, 9), 8, 3, 1), ((2, 4, 9, 9), 6, 3, 2)]:
    rng = np.random.default_rng(1)
    x = rng.standard_normal(xs).astype(np.float32)
    w = rng.standard_normal((co, xs[1] // g, k, k)).astype(np.float32)
    b = np.zeros(co, np.float32)
    d = ops.conv_desc(xs, co, k, 1, 0, 1, g)
    y = torch.empty((xs[0], co, d.out_h, d.out_w), device=dev)
    ops.conv2d_fwd(d, torch.from_numpy(x).to(dev), torch.from_numpy(w).to(dev), torch.from_numpy(b).to(dev), y)
    yt = torch.nn.functional.conv2d(torch.from_numpy(x), torch.from_numpy(w), groups=g).numpy()
    err = np.abs(y.cpu().numpy() - yt).max(axis=(0, 2, 3))
    print(xs, co, k, g, "per-channel max err:", np.round(err, 4).tolist())
    # single-weight probes: which weight entries does channel m actually use?
    K = w[0].size
    for m in [0, co - 1]:
        used = []
        for kk in range(K):
            w2 = np.zeros_like(w); w2.reshape(co, K)[m, kk] = 1.0
            ops.conv2d_fwd(d, torch.from_numpy(x).to(dev), torch.from_numpy(w2).to(dev), torch.from_numpy(b).to(dev), y)
            yt = torch.nn.functional.conv2d(torch.from_numpy(x), torch.from_numpy(w2), groups=g).numpy()
            if np.abs(y.cpu().numpy() - yt).max() > 1e-4: used.append(kk)
        print("  channel", m, "wrong when only weight k is set:", used)
