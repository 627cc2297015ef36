"""Diagnostic: per-group cycle shares of k_conv_cb16_x6 (AlexNet conv2's
5x5 form and the conv3 / conv4 / conv5 3x3 forms at b256) from the stamp build
(make VARIANT=-DRRAM_CB_STAMP LIBDIR=lib_cbstamp; RRAM_LIB_DIR points at it).
Prints, per slot, the mean s_memtime cycles per wave per tile; the stamps'
own cost (~40-200 cycles each, and each drains the wave's LDS reads) is
included, so read shares, not lengths."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rram-caffe-simulation_amd" / "python"))
import torch  # noqa: E402
from rramsim import ops  # noqa: E402
from rramsim._kernels import load  # noqa: E402

lib = load()
lib.rram_debug_cb_stamps.argtypes = [C.c_void_p, C.c_int]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1)
for name, cin, cout, grp, k, hw in (("conv2", 96, 256, 2, 5, 27), ("conv3", 256, 384, 1, 3, 13),
                                    ("conv4", 384, 384, 2, 3, 13), ("conv5", 384, 256, 2, 3, 13)):
    H = k * k // 2                 # pair groups per K-tile
    names = [f"even g{j}" for j in range(H)] + ["odd cross"] + [f"odd g{j}" for j in range(H)] + \
            ["bar K-tile end", "bar cross", "prologue", "epilogue"]
    x = torch.randn(256, cin, hw, hw, device=dev, generator=g)
    w = torch.randn(cout, cin // grp, k, k, device=dev, generator=g) * 0.02
    b = torch.zeros(cout, device=dev)
    d = ops.conv_desc(tuple(x.shape), cout, k, 1, k // 2, 1, grp)
    y = torch.empty((256, cout, hw, hw), device=dev)
    for _ in range(3):
        ops.conv2d_fwd(d, x, w, b, y, relu=True)
    torch.cuda.synchronize()
    lib.rram_debug_cb_stamps(None, 64)
    reps = 10
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        ops.conv2d_fwd(d, x, w, b, y, relu=True)
    e.record()
    torch.cuda.synchronize()
    out = (C.c_ulonglong * 64)()
    lib.rram_debug_cb_stamps(out, 64)
    n = 2 * H + 5
    tiles = out[n]
    tot = sum(out[k] for k in range(n))
    print(f"{name}: call {s.elapsed_time(e) / reps * 1e3:.1f} us (stamp build, incl. the input pack), "
          f"wave-tiles {tiles}, plan {ops.conv_octet_plan(d)}")
    for k in range(n):
        print(f"  {names[k]:15s} {out[k] / max(tiles, 1):9.0f} cyc/tile  {100 * out[k] / tot:5.1f} %")
    print(f"  total {tot / max(tiles, 1):.0f} cycles per wave-tile")
