"""CPU tests of the drop-in boundary: the C-ABI libraries load and export every
symbol their headers declare (no compute calls — there is no GPU here)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared(header: Path):
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rram_[a-z0-9_]+)\s*\(", text)))


def test_kernel_header_symbols_exported():
    from rramsim import _kernels as K
    lib = K.load()
    names = declared(ROOT / "include" / "rram_kernels.h")
    assert len(names) > 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # every declared symbol has a ctypes signature (the Python view is complete)
    assert sorted(set(names) - set(K.SIGNATURES)) == []


def test_kernel_structs_match_header():
    from rramsim import _kernels as K
    assert ctypes.sizeof(K.InjectCfg) == 56
    assert ctypes.sizeof(K.InjectSeg) == 8 + 8 + 8 + 4 + 4 + 56
    assert ctypes.sizeof(K.FailSeg) == 40
    # 5 pointers, n, 3 floats + int, counter pointer, flipped-kernel pointer + 4 ints
    assert ctypes.sizeof(K.UpdateSeg) == 5 * 8 + 8 + 4 * 4 + 8 + 8 + 4 * 4
    assert K.UpdateSeg.broken_count.offset == 64
    assert K.UpdateSeg.w_flip.offset == 72 and K.UpdateSeg.flip_taps.offset == 92
    assert ctypes.sizeof(K.ConvDesc) == 16 * 4


def test_version_and_error_string_callable():
    from rramsim import _kernels as K
    lib = K.load()
    assert lib.rram_kernels_version().startswith(b"rram_kernels")
    assert isinstance(lib.rram_last_error(), bytes)


def test_invalid_args_return_status_not_abort():
    """Argument validation runs on the host before any launch (no GPU needed)."""
    from rramsim import _kernels as K
    lib = K.load()
    assert lib.rram_fail_apply(None, None, None, None, -1, 100.0, 1e-20, None, None) == K.RRAM_EINVAL
    assert b"n < 0" in lib.rram_last_error()
    assert lib.rram_inject_rng(None, None, 10, None, 0, 0, 0, None, None) == K.RRAM_EINVAL
    d = K.ConvDesc(1, 3, 8, 8, 4, 3, 3, 0, 0, 1, 1, 1, 1, 2, 0, 0)   # 3 % 2 != 0
    assert lib.rram_conv_out_shape(ctypes.byref(d)) == K.RRAM_EINVAL
    d = K.ConvDesc(2, 3, 227, 227, 96, 11, 11, 0, 0, 4, 4, 1, 1, 1, 0, 0)
    assert lib.rram_conv_out_shape(ctypes.byref(d)) == K.RRAM_OK and d.out_h == 55 == d.out_w
    seg = K.UpdateSeg(None, None, None, None, None, -1, 0.0, 0.0, 0.0, 0, None)
    assert lib.rram_fused_update_fail_batched(ctypes.byref(seg), 1, 0.9, 100.0, 1e-20, None) == K.RRAM_EINVAL
    assert lib.rram_fused_update_fail_batched(None, 33, 0.9, 100.0, 1e-20, None) == K.RRAM_EINVAL
    # a flipped-kernel destination whose geometry does not cover the segment
    seg = K.UpdateSeg(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16), None, None, 100, 0.0, 0.0, 0.0, 0,
                      None, ctypes.c_void_p(16), 2, 3, 4, 9)
    assert lib.rram_fused_update_fail_batched(ctypes.byref(seg), 1, 0.9, 100.0, 1e-20, None) == K.RRAM_EINVAL
    assert b"flip geometry" in lib.rram_last_error()
    # the flipped-kernel data gradient serves stride 1 with padding <= dil (k - 1) only
    d = K.ConvDesc(8, 32, 16, 16, 32, 5, 5, 2, 2, 1, 1, 1, 1, 1, 0, 0)
    assert lib.rram_conv2d_flip_applies(ctypes.byref(d)) == 1
    d = K.ConvDesc(8, 3, 227, 227, 96, 11, 11, 0, 0, 4, 4, 1, 1, 1, 0, 0)
    assert lib.rram_conv2d_flip_applies(ctypes.byref(d)) == 0
    d = K.ConvDesc(8, 32, 16, 16, 32, 3, 3, 3, 3, 1, 1, 1, 1, 1, 0, 0)   # pad 3 > k - 1
    assert lib.rram_conv2d_flip_applies(ctypes.byref(d)) == 0
    assert lib.rram_conv2d_flip_applies(None) == 0
    # zero-size work is a successful no-op that never touches the device
    assert lib.rram_fail_apply(None, None, None, None, 0, 100.0, 1e-20, None, None) == K.RRAM_OK


def test_caffe_header_symbols_exported():
    hdr = ROOT / "include" / "rram_caffe.h"
    if not hdr.exists():
        pytest.skip("host runtime header not present yet")
    from rramsim import _kernels as K
    K.load()
    lib = ctypes.CDLL(str(K.CAFFE_SO))
    missing = [n for n in declared(hdr) if not hasattr(lib, n)]
    assert not missing, missing


def test_engine_plans_host_side():
    """The engine / kernel plans are host logic (no GPU): AlexNet conv2-5 at
    b256 take the channel-octet kernel (their inputs would read an octet
    companion), conv1 the wide bf16x6 kernel, and shapes outside the octet
    kernel's range (Cin/group % 16 != 0, stride 2, 7x7, 1x1) do not."""
    from rramsim import ops
    octet = [((256, 96, 27, 27), 256, 5, 2, 2), ((256, 256, 13, 13), 384, 3, 1, 1),
             ((256, 384, 13, 13), 384, 3, 1, 2), ((256, 384, 13, 13), 256, 3, 1, 2),
             ((8, 64, 28, 28), 128, 3, 1, 1)]
    for x, cout, k, p, g in octet:
        d = ops.conv_desc(x, cout, k, 1, p, 1, g)
        assert ops.conv_input_octets(d) == 1, (x, cout, k)
        assert ops.f32_engine_for_conv(d) == ops.ENGINE_BF16X6
    not_octet = [((256, 3, 227, 227), 96, 11, 0, 1, 4), ((4, 24, 28, 28), 64, 3, 1, 1, 1),
                 ((4, 64, 28, 28), 64, 3, 1, 1, 2), ((4, 3, 224, 224), 64, 7, 3, 1, 2),
                 ((4, 64, 28, 28), 64, 1, 0, 1, 1)]
    for x, cout, k, p, g, s in not_octet:
        d = ops.conv_desc(x, cout, k, s, p, 1, g)
        assert ops.conv_input_octets(d) == 0, (x, cout, k, s)
    conv1 = ops.conv_desc((256, 3, 227, 227), 96, 11, 4, 0, 1, 1)
    assert ops.f32_engine_for_conv(conv1) == ops.ENGINE_BF16X6
    prev = ops.set_f32_engine(ops.ENGINE_F32)
    try:
        assert ops.conv_input_octets(ops.conv_desc(*octet[0][:2], 5, 1, 2, 1, 2)) == 0
        assert ops.f32_engine_for_conv(conv1) == ops.ENGINE_F32
    finally:
        ops.set_f32_engine(prev)


def test_engine_plans_round6_host_side():
    """Round-6 plans (host logic, no GPU): GoogLeNet conv2 on row-aligned
    64 x 128 per-image tiles (28 per 56 x 56 image), the 7 x 7 stage's 3x3 /
    5x5 on whole-image tiles, GoogLeNet conv1 (7x7 / 2, 3 channels) on the
    bf16x6 engine without an octet input, the 1x1 reductions' companion-only
    epilogue; and shapes whose outputs the 32-bit epilogue offsets cannot
    address fall back to the fp32 engine."""
    from rramsim import ops
    pl = ops.conv_octet_plan(ops.conv_desc((256, 64, 56, 56), 192, 3, 1, 1, 1, 1))
    assert {k: pl[k] for k in ("rows", "cols", "per_cu", "tiles_per_image")} == \
        dict(rows=64, cols=128, per_cu=2, tiles_per_image=28), pl
    for x, cout, k, p in [((256, 192, 7, 7), 384, 3, 1), ((256, 160, 7, 7), 320, 3, 1), ((256, 48, 7, 7), 128, 5, 2)]:
        pl = ops.conv_octet_plan(ops.conv_desc(x, cout, k, 1, p, 1, 1))
        assert pl is not None and pl["per_cu"] == 2 and pl["tiles_per_image"] == 0, (x, pl)
    c1 = ops.conv_desc((256, 3, 224, 224), 64, 7, 2, 3, 1, 1)
    assert ops.f32_engine_for_conv(c1) == ops.ENGINE_BF16X6 and ops.conv_input_octets(c1) == 0
    assert ops.conv_output_octets_only(ops.conv_desc((256, 192, 28, 28), 96, 1, 1, 0, 1, 1)) == 1
    assert ops.conv_output_octets_only(ops.conv_desc((256, 192, 28, 28), 20, 1, 1, 0, 1, 1)) == 0  # partial octet
    for x, cout, k, s, p, g in [((4096, 96, 27, 27), 256, 5, 1, 2, 2), ((2048, 3, 227, 227), 96, 11, 4, 0, 1)]:
        d = ops.conv_desc(x, cout, k, s, p, 1, g)
        assert ops.f32_engine_for_conv(d) == ops.ENGINE_F32, x


def test_octet_kernel_tile_plans_host_side():
    """The channel-octet kernel's tile plans for AlexNet b256 (host logic, no
    GPU): every layer at two workgroups per CU (16x16x32 form):
    conv2's 5x5 on 128 x 128 per-image tiles (its contiguous 128 x 128 tiles
    spanning two images would need more than 8 LDS pieces), conv3 and conv5
    on contiguous 128 x 128 tiles, conv4 (192 rows per group) on contiguous
    64 x 128 tiles (128-row tiles would pad a quarter of its rows)."""
    from rramsim import ops
    want = {"conv2": (((256, 96, 27, 27), 256, 5, 2, 2), dict(rows=128, cols=128, per_cu=2, tiles_per_image=6)),
            "conv3": (((256, 256, 13, 13), 384, 3, 1, 1), dict(rows=128, cols=128, per_cu=2, tiles_per_image=0)),
            "conv4": (((256, 384, 13, 13), 384, 3, 1, 2), dict(rows=64, cols=128, per_cu=2, tiles_per_image=0)),
            "conv5": (((256, 384, 13, 13), 256, 3, 1, 2), dict(rows=128, cols=128, per_cu=2, tiles_per_image=0))}
    for name, ((x, cout, k, p, g), exp) in want.items():
        pl = ops.conv_octet_plan(ops.conv_desc(x, cout, k, 1, p, 1, g))
        assert pl is not None, name
        assert {kk: pl[kk] for kk in exp} == exp, (name, pl)
        if pl["per_cu"] == 2:
            assert pl["pieces"] <= 8, (name, pl)     # 2 x 8 x 4 KB LDS stages per workgroup
    assert ops.conv_octet_plan(ops.conv_desc((256, 3, 227, 227), 96, 11, 4, 0, 1, 1)) is None
