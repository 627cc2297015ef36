"""Diagnostic: per-group cycle shares of k_conv1_ring_x6 from the stamp build
(make VARIANT=-DRRAM_C1_STAMP LIBDIR=lib_c1stamp; RRAM_LIB_DIR points at it).
Prints, per slot, the mean s_memtime cycles per wave per tile; the stamps'
own cost (~40 cycles each) is included, so read shares, not lengths."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))
import torch  # noqa: E402
from rramsim import ops  # noqa: E402
from rramsim._kernels import load  # noqa: E402

lib = load()
lib.rram_debug_c1_stamps.argtypes = [C.c_void_p, C.c_int]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randint(0, 256, (256, 3, 227, 227), device=dev, generator=g).float() - 128
w = torch.randn(96, 3, 11, 11, device=dev, generator=g) * 0.01
b = torch.zeros(96, device=dev)
d = ops.conv_desc(tuple(x.shape), 96, 11, 4, 0, 1, 1)
y = torch.empty((256, 96, d.out_h, d.out_w), device=dev)
for _ in range(5):
    ops.conv2d_fwd(d, x, w, b, y, relu=True)
torch.cuda.synchronize()
lib.rram_debug_c1_stamps(None, 64)
reps = 20
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    ops.conv2d_fwd(d, x, w, b, y, relu=True)
e.record()
torch.cuda.synchronize()
out = (C.c_ulonglong * 64)()
lib.rram_debug_c1_stamps(out, 64)
G = 25
tiles = out[G + 4]
print(f"kernel {s.elapsed_time(e) / reps * 1e3:.1f} us (stamp build), wave-tiles {tiles}")
tot = sum(out[k] for k in range(G + 4))
for k in range(G + 4):
    name = f"group {k}" if k < G else ["barrier ch0", "barrier ch1", "barrier end", "tile setup"][k - G]
    print(f"{name:12s} {out[k] / max(tiles, 1):8.0f} cyc/tile  {100 * out[k] / tot:5.1f} %")
print(f"total {tot / max(tiles, 1):.0f} cycles per wave-tile")
