"""CPU tests: the oracle pinned against the golden vectors / reference KATs,
and two independent restatements cross-checked (C oracle vs numpy)."""
import json
import math
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden"


def from_bits(b):
    return np.array(b, np.uint32).view(np.float32)


# -------------------------------------------------------------------- Philox
def test_philox_random123_kat(oracle_mod):
    # Random123 kat_vectors, philox4x32 R=10
    assert oracle_mod.philox([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert oracle_mod.philox([0xffffffff] * 4, [0xffffffff] * 2) == \
        [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert oracle_mod.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
                             [0xa4093822, 0x299f31d0]) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


# ---------------------------------------------------------------- fail_apply
def test_fail_apply_golden(oracle_mod):
    d = json.loads((GOLD / "fail_apply_kat.json").read_text())
    for c in d["cases"]:
        w, e, v = from_bits(c["w0_bits"]), from_bits(c["e0_bits"]), from_bits(c["v_bits"])
        nb = None
        for st in c["steps"]:
            w, e, nb = oracle_mod.fail_apply(from_bits(st["dw_bits"]), w, e, v, d["decrement"], d["eps"])
        assert np.array_equal(w.view(np.uint32), np.array(c["w_bits"], np.uint32)), c["k"]
        assert np.array_equal(e.view(np.uint32), np.array(c["e_bits"], np.uint32)), c["k"]
        assert nb == c["broken"]


def test_fail_apply_fp32_inexact_decrement(oracle_mod):
    # Appendix A Q1: 1e8 - 100 in fp32 is 99,999,904
    w, e, _ = oracle_mod.fail_apply([1.0], [0.5], [1e8], [1.0])
    assert e[0] == np.float32(99999904.0) and w[0] == np.float32(0.5)


def test_fault_threshold_golden(oracle_mod):
    d = json.loads((GOLD / "threshold_kat.json").read_text())
    out = oracle_mod.fault_threshold(from_bits(d["u_bits"]), d["split1"], d["split2"])
    assert np.array_equal(out.view(np.uint32), np.array(d["v_bits"], np.uint32))


# --------------------------------------------------------------------- GEMM
def test_gemm_kat_all_transposes(oracle_mod):
    d = json.loads((GOLD / "gemm_kat.json").read_text())
    C = np.array(d["C"], np.float32).reshape(2, 4)
    A, B, AT, BT = (np.array(d[k], np.float32) for k in ("A", "B", "A_T", "B_T"))
    assert np.array_equal(oracle_mod.gemm(0, 0, 2, 4, 3, 1.0, A, B), C)
    assert np.array_equal(oracle_mod.gemm(1, 0, 2, 4, 3, 1.0, AT, B), C)
    assert np.array_equal(oracle_mod.gemm(1, 1, 2, 4, 3, 1.0, AT, BT), C)
    assert np.array_equal(oracle_mod.gemm(0, 1, 2, 4, 3, 1.0, A, BT), C)


def test_gemm_alpha_beta(oracle_mod):
    rng = np.random.default_rng(1701)
    A, B, C0 = rng.standard_normal((5, 7)), rng.standard_normal((7, 3)), rng.standard_normal((5, 3))
    out = oracle_mod.gemm(0, 0, 5, 3, 7, 0.5, A, B, 2.0, C0)
    np.testing.assert_allclose(out, 0.5 * A @ B + 2.0 * C0, rtol=1e-5, atol=1e-5)


# -------------------------------------------------------------- conv/im2col
CONV_CASES = [  # test_convolution_layer.cpp shapes: bottom 2x3x6x4
    dict(x=(2, 3, 6, 4), cout=4, k=3, s=2, p=0, d=1, g=1),   # TestSimpleConvolution
    dict(x=(2, 3, 6, 4), cout=3, k=3, s=2, p=0, d=1, g=3),   # TestSimpleConvolutionGroup
    dict(x=(2, 3, 6, 4), cout=4, k=1, s=1, p=0, d=1, g=1),   # Test1x1Convolution
    dict(x=(2, 3, 8, 7), cout=4, k=3, s=1, p=0, d=2, g=1),   # TestDilatedConvolution
    dict(x=(2, 3, 6, 4), cout=4, k=3, s=1, p=1, d=1, g=1),   # padded
    dict(x=(1, 3, 31, 31), cout=8, k=11, s=4, p=0, d=1, g=1),  # AlexNet conv1 geometry
    dict(x=(1, 8, 13, 13), cout=8, k=3, s=1, p=1, d=1, g=2),   # AlexNet conv4 geometry
]


@pytest.mark.parametrize("cs", CONV_CASES)
def test_conv_naive_vs_im2col(oracle_mod, cs):
    rng = np.random.default_rng(1701)
    x = rng.standard_normal(cs["x"]).astype(np.float32)
    w = rng.standard_normal((cs["cout"], cs["x"][1] // cs["g"], cs["k"], cs["k"])).astype(np.float32)
    b = rng.standard_normal(cs["cout"]).astype(np.float32)
    a = oracle_mod.conv_naive(x, w, b, cs["s"], cs["p"], cs["d"], cs["g"])
    c = oracle_mod.conv_im2col(x, w, b, cs["s"], cs["p"], cs["d"], cs["g"])
    np.testing.assert_allclose(a, c, atol=1e-4, rtol=1e-4)  # test_convolution_layer.cpp:256


def test_im2col_c_vs_numpy_and_adjoint(oracle_mod):
    rng = np.random.default_rng(3)
    im = rng.standard_normal((5, 15, 15)).astype(np.float32)  # test_im2col_kernel.cu:36-62 shape
    for (k, p, s, d) in [(3, 0, 2, 3), (3, 1, 1, 1), (5, 2, 3, 1)]:
        c1 = oracle_mod.im2col(im, k, k, p, p, s, s, d, d)
        c2 = oracle_mod.im2col_np(im, k, k, p, p, s, s, d, d)
        assert np.array_equal(c1, c2)
        col = rng.standard_normal(c1.shape).astype(np.float32)
        back = oracle_mod.col2im(col, 5, 15, 15, k, k, p, p, s, s, d, d)
        lhs = float(np.dot(col.ravel().astype(np.float64), c1.ravel()))
        rhs = float(np.dot(back.ravel().astype(np.float64), im.ravel()))
        assert abs(lhs - rhs) <= 1e-3 * max(1.0, abs(lhs))


# ---------------------------------------------------------------- injection
def _ci(n, p, z=3.8):
    # test_random_number_generator.cpp:17-19,53-55: 3.8 sigma bound
    return z * math.sqrt(p * (1 - p) / n)


def test_inject_binomial_ci(oracle_mod):
    from rramsim import make_inject_cfg
    n = 200_000
    src = np.linspace(-1, 1, n, dtype=np.float32)
    for p in (0.001, 0.05, 0.10):
        c = make_inject_cfg(p, 5, 90, 5)
        cfg = oracle_mod.InjectCfg(c.thr_fault, c.thr_neg, c.thr_zero, c.thr_sa1, 1.0, 0.0, 0, 0.0, 0, 0)
        dst, nb = oracle_mod.inject(src, cfg, seed=1701, map_id=7, layer_id=3)
        changed = dst != src
        assert abs(nb / n - p) <= _ci(n, p)
        broken_vals = dst[np.isin(dst, [-1, 0, 1]) & changed]
        if nb > 2000:
            frac_zero = np.mean(broken_vals == 0)
            assert abs(frac_zero - 0.9) <= _ci(len(broken_vals), 0.9) + 0.01


def test_inject_quantised_on_grid(oracle_mod):
    from rramsim import make_inject_cfg
    src = np.random.default_rng(5).uniform(-0.5, 0.5, 10001).astype(np.float32)
    c = make_inject_cfg(0.0, quant_levels=16, g_max=0.5)
    cfg = oracle_mod.InjectCfg(c.thr_fault, c.thr_neg, c.thr_zero, c.thr_sa1, 1.0, 0.5, 16, 0.0, 0, 0)
    dst, nb = oracle_mod.inject(src, cfg, 1, 0, 0)
    assert nb == 0
    delta = np.float32(1.0) / np.float32(15)
    t = (dst + 0.5) / delta
    assert np.max(np.abs(t - np.round(t))) < 1e-3
    assert np.max(np.abs(dst - src)) <= delta / 2 + 1e-6


def test_fault_init_rate_matches_gaussian(oracle_mod):
    from rramsim import gaussian_fault_rate, split_thresholds
    n = 100_000
    mean, std = 2000.0, 1000.0                        # P(e <= 0) = Phi(-2) = 2.28 %
    tn, tz = split_thresholds(10, 20, 10)
    e, v = oracle_mod.fault_init(n, mean, std, tn, tz, seed=1701)
    p = gaussian_fault_rate(mean, std)
    assert abs(np.mean(e <= 0) - p) <= _ci(n, p)
    assert abs(np.mean(e) - mean) < 4 * std / math.sqrt(n)
    assert abs(np.std(e) - std) < 0.02 * std
    for val, q in ((-1, 0.25), (0, 0.5), (1, 0.25)):
        assert abs(np.mean(v == val) - q) <= _ci(n, q)


# ----------------------------------------------------------- host helpers
def test_split_thresholds_exact():
    from rramsim import split_thresholds, prob_threshold
    tn, tz = split_thresholds(10, 20, 10)
    assert tn == 1 << 30 and tz == 3 << 30
    assert split_thresholds(5, 90, 5) == (-(-5 * 2**32 // 100), -(-95 * 2**32 // 100))
    assert prob_threshold(0.0) == 0 and prob_threshold(1.0) == 2**32
    with pytest.raises(ValueError):
        split_thresholds(-1, 1, 1)


def test_threshold_strategy_oracle(oracle_mod):
    dw = np.array([0.0, 1e-4, -1e-3, 1e-3, 0.5, -2e-3], np.float32)
    out, n = oracle_mod.threshold(dw, 1e-3)
    assert n == 4 and np.array_equal(out, np.array([0, 0, 0, 0, 0.5, -2e-3], np.float32))


def test_pool_out_rule(oracle_mod):
    # AlexNet pool1: 55 -> 27 (k3 s2); GoogLeNet pool1/3x3_s2: 112 -> 56 (ceil)
    assert oracle_mod.pool_out(55, 3, 0, 2) == 27
    assert oracle_mod.pool_out(112, 3, 0, 2) == 56
    assert oracle_mod.pool_out(7, 3, 1, 2) == 4


def test_caffe_cpu_restatement_matches_numpy_oracle():
    """oracle/caffe_cpu.c (bench.py's CPU baseline) computes the same layers as
    the numpy restatements: conv (per-image im2col + group sgemm + bias sgemm),
    IP, ReLU, cross-channel LRN, MAX pooling, softmax."""
    import numpy as np
    import oracle
    oracle.cc_init(2)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((3, 8, 15, 13)).astype(np.float32)
    for (co, k, s, p, g) in ((6, 3, 1, 1, 1), (8, 5, 2, 2, 2), (4, 1, 1, 0, 1), (6, 3, 2, 0, 2)):
        w = rng.standard_normal((co, 8 // g, k, k)).astype(np.float32)
        b = rng.standard_normal(co).astype(np.float32)
        np.testing.assert_allclose(oracle.cc_conv(x, w, b, s, p, g), oracle.conv_naive(x, w, b, s, p, 1, g),
                                   rtol=1e-5, atol=1e-5)
    xi = rng.standard_normal((5, 40)).astype(np.float32)
    wi = rng.standard_normal((7, 40)).astype(np.float32)
    bi = rng.standard_normal(7).astype(np.float32)
    np.testing.assert_allclose(oracle.cc_ip(xi, wi, bi), xi @ wi.T + bi, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(oracle.cc_relu(x.copy()), oracle.relu(x))
    np.testing.assert_allclose(oracle.cc_lrn(x, 5, 1e-4, 0.75), oracle.lrn(x, 5, 1e-4, 0.75), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(oracle.cc_maxpool(x, 3, 2), oracle.pool(x, 3, 2))
    np.testing.assert_allclose(oracle.cc_softmax(xi), oracle.softmax(xi), rtol=1e-5, atol=1e-7)


def test_caffe_cpu_alexnet_map_small():
    """The CPU-baseline pipeline runs end to end (2 images) and its fault map
    breaks ~p of the 58.6M IP cells (3.8 sigma binomial bound)."""
    import math
    import oracle
    t, meta = oracle.caffe_cpu_alexnet_map(batch=256, images=2, threads=2, p_fault=0.01)
    n = 58_631_144
    assert abs(meta["broken_cells"] / n - 0.01) <= 3.8 * math.sqrt(0.01 * 0.99 / n)
    assert meta["finite"] and {"conv1", "fc8", "norm1", "pool5"} <= set(t)
