"""Developer probe: C4 graph training with rram_release_caches between step()
calls; prints which iteration fails (if any)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))
import torch  # noqa: E402
from rramsim import caffe, models, kernels  # noqa: E402

torch.cuda.set_device(0)
caffe.set_stream_from_torch()
caffe.set_random_seed(1701)
sp = models.solver(base_lr=0.001, momentum=0.9, weight_decay=0.004, lr_policy="fixed", max_iter=1000,
                   failure_mean=5e4, failure_std=1.5e4, failure_prob=(5, 90, 5), threshold=0.001)
s = caffe.Solver(sp, models.cifar10_full(train_batch=20, test_batch=20),
                 dict(models.net_options("cifar10_full"), fused_update=True))
s.set_graph(True)
for n in [3, 1, 1, 1, 2]:
    for _ in range(n):
        try:
            s.step(1)
            print("iter ok", s.iter, "graph", s.graph_active(), flush=True)
        except Exception as e:
            print("iter FAILED at", s.iter, e, flush=True)
            raise SystemExit(1)
    torch.cuda.synchronize()
    kernels.check(kernels.load().rram_release_caches(), "release")
    print("released", flush=True)
