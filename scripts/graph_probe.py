"""Probe: one MC map (injection + AlexNet b256 forward + accumulation) replayed
as a captured HIP graph vs launched eagerly, to price the launch gaps.  The
replayed graph repeats the same map id (same work); not a bench line."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))
import torch  # noqa: E402
from rramsim import caffe, make_inject_cfg, models  # noqa: E402

torch.cuda.set_device(0)
caffe.set_stream_from_torch()
caffe.set_random_seed(1701)
net = caffe.Net(models.alexnet(test_batch=256), "test", models.net_options("alexnet"))
mc = caffe.MonteCarlo(net, make_inject_cfg(0.01), seed=1701, max_maps=400)
for i in range(30):
    mc.run(i, 1)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    for i in range(40):
        mc.run(100 + i, 1)
    torch.cuda.synchronize()
    print(f"eager  {(time.perf_counter() - t0) / 40 * 1e3:.3f} ms/map", flush=True)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    caffe.set_stream_from_torch()
    mc.run(200, 1)            # warm on the side stream
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        caffe.set_stream_from_torch()
        mc.run(201, 1)
caffe.set_stream_from_torch()
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    for i in range(40):
        g.replay()
    torch.cuda.synchronize()
    print(f"graph  {(time.perf_counter() - t0) / 40 * 1e3:.3f} ms/map", flush=True)
for rep in range(2):
    t0 = time.perf_counter()
    for i in range(40):
        mc.run(300 + i, 1)
    torch.cuda.synchronize()
    print(f"eager  {(time.perf_counter() - t0) / 40 * 1e3:.3f} ms/map", flush=True)
