"""Debug probes for the conv1 bf16x6 kernel (developer tool)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from rramsim import ops  # noqa: E402

dev = torch.device("cuda", 0)
d = ops.conv_desc((1, 3, 227, 227), 96, 11, 4, 0, 1, 1)
y = torch.empty(1, 96, 55, 55, device=dev)
def run(x, w, name):
    ops.conv2d_fwd(d, x, w, None, y)
    torch.cuda.synchronize()
    ref = F.conv2d(x.double(), w.double(), None, stride=4)
    dif = (y.double() - ref).abs()
    print(name, "max|d|", float(dif.max()), "y[0,0,0,:6]", y[0, 0, 0, :6].tolist(), "ref", ref[0, 0, 0, :6].tolist(),
          "bad rows(oh)", (dif[0].amax(dim=(0, 2)) > 1e-3).nonzero().flatten().tolist()[:12],
          "bad cols(ow)", (dif[0].amax(dim=(0, 1)) > 1e-3).nonzero().flatten().tolist()[:12],
          "bad m", (dif[0].amax(dim=(1, 2)) > 1e-3).nonzero().flatten().tolist()[:12])
ones = torch.ones(1, 3, 227, 227, device=dev)
run(ones, torch.ones(96, 3, 11, 11, device=dev), "x=1 w=1")
for c in range(3):
    w = torch.zeros(96, 3, 11, 11, device=dev); w[:, c] = 1
    run(ones, w, f"x=1 w=1 ch{c}")
for kh in (0, 5, 6, 10):
    w = torch.zeros(96, 3, 11, 11, device=dev); w[:, 0, kh] = 1
    run(ones, w, f"w row {kh}")
for kw in (0, 3, 4, 10):
    w = torch.zeros(96, 3, 11, 11, device=dev); w[:, 0, :, kw] = 1
    run(ones, w, f"w col {kw}")
xr = torch.arange(227, device=dev, dtype=torch.float32).repeat(1, 3, 227, 1)
w = torch.zeros(96, 3, 11, 11, device=dev); w[:, 0, 0, 0] = 1
run(xr, w, "x=col idx, w[0,0,0]=1")
xr = torch.arange(227, device=dev, dtype=torch.float32).reshape(227, 1).repeat(1, 3, 1, 227)
run(xr, w, "x=row idx, w[0,0,0]=1")
