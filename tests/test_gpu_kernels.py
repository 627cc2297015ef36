"""GPU parity tests: the HIP kernels through the C-ABI vs the CPU oracle.

Bit-exact for mask application, endurance arithmetic, quantisation and the
integer RNG decisions; fp32 tolerance (stated per test) for floating-point
contractions and transcendental-based draws.
"""
import json
import math
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def from_bits(b):
    return np.array(b, np.uint32).view(np.float32)


def T(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)


def N(t):
    import torch
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float32).view(np.uint32),
                          np.asarray(b, np.float32).view(np.uint32))


# ------------------------------------------------------------- fail_apply
def test_fail_apply_golden_bit_exact(device):
    from rramsim import ops
    d = json.loads((GOLD / "fail_apply_kat.json").read_text())
    for c in d["cases"]:
        w, e, v = T(from_bits(c["w0_bits"]), device), T(from_bits(c["e0_bits"]), device), \
            T(from_bits(c["v_bits"]), device)
        cnt = ops.counters(1, device)
        for st in c["steps"]:
            cnt.zero_()
            ops.fail_apply(T(from_bits(st["dw_bits"]), device), w, e, v, d["decrement"], d["eps"], cnt)
        assert bits_equal(N(w), from_bits(c["w_bits"]))
        assert bits_equal(N(e), from_bits(c["e_bits"]))
        assert int(N(cnt)[0]) == c["broken"]


@pytest.mark.parametrize("n", [0, 1, 3, 4097, 1 << 20, 3_000_001])
def test_fail_apply_random_vs_oracle(device, oracle_mod, n):
    from rramsim import ops
    rng = np.random.default_rng(n)
    e = rng.normal(300, 200, n).astype(np.float32)
    v = rng.integers(-1, 2, n).astype(np.float32)
    w = rng.standard_normal(n).astype(np.float32)
    dw = np.where(rng.random(n) < 0.3, 0.0, rng.standard_normal(n) * 1e-3).astype(np.float32)
    tw, te = T(w, device), T(e, device)
    cnt = ops.counters(1, device)
    for _ in range(3):
        cnt.zero_()
        ops.fail_apply(T(dw, device), tw, te, T(v, device), counter=cnt)
        w, e, nb = oracle_mod.fail_apply(dw, w, e, v)
    assert bits_equal(N(tw), w) and bits_equal(N(te), e) and int(N(cnt)[0]) == nb


def test_fail_apply_beyond_2e31_elements(device, oracle_mod):
    """Maximum size: Fail() over one blob of 2^31 + 4099 cells (4 x 8.6 GB,
    int64 addressing past 2^31).  Windows at the start, across 2^31 and at the
    ragged tail match the oracle bit for bit (Fail is element-wise); the
    broken counter equals the number of cells left at endurance <= 0."""
    import torch
    from rramsim import ops
    n = (1 << 31) + 4099
    g = torch.Generator(device=device).manual_seed(3)
    e = torch.randn(n, device=device, generator=g).mul_(150).add_(120)
    v = torch.randint(-1, 2, (n,), device=device, generator=g).float()
    w = torch.randn(n, device=device, generator=g)
    dw = torch.randn(n, device=device, generator=g).mul_(1e-3)
    dw[::3] = 0.0
    wins = [(lo, min(n, lo + 1003)) for lo in (0, (1 << 31) - 1000, n - 1003)]
    before = [tuple(N(t[lo:hi]).copy() for t in (dw, w, e, v)) for lo, hi in wins]
    cnt = ops.counters(1, device)
    ops.fail_apply(dw, w, e, v, counter=cnt)
    torch.cuda.synchronize()
    for (lo, hi), (dw0, w0, e0, v0) in zip(wins, before):
        w1, e1, _ = oracle_mod.fail_apply(dw0, w0, e0, v0)
        assert bits_equal(N(w[lo:hi]), w1) and bits_equal(N(e[lo:hi]), e1), lo
    assert int(N(cnt)[0]) == int((e <= 0).sum().item())
    del e, v, w, dw
    torch.cuda.empty_cache()


def test_fail_apply_batched_unaligned_segments(device, oracle_mod):
    """Segments at odd float offsets of one flat buffer (the P2PSync-style
    aliasing of params, parallel.cpp:25-67) take the scalar path; an empty
    segment (a zero-size blob) in the middle is skipped and counts 0."""
    import torch
    from rramsim import ops
    rng = np.random.default_rng(9)
    sizes = [4096 * 9, 4096, 0, 1001, 1000, 37, 1]
    tot = sum(sizes) + 1
    e = rng.normal(150, 100, tot).astype(np.float32)
    v = rng.integers(-1, 2, tot).astype(np.float32)
    w = rng.standard_normal(tot).astype(np.float32)
    dw = rng.standard_normal(tot).astype(np.float32)
    te, tv, tw, tdw = (T(a, device) for a in (e, v, w, dw))
    segs, off = [], 1
    for s in sizes:
        segs.append((tdw[off:off + s], tw[off:off + s], te[off:off + s], tv[off:off + s]))
        off += s
    cnt = ops.counters(len(sizes), device)
    ops.fail_apply_batched(segs, counters_t=cnt)
    off = 1
    for i, s in enumerate(sizes):
        sl = slice(off, off + s)
        w2, e2, nb = oracle_mod.fail_apply(dw[sl], w[sl], e[sl], v[sl])
        w[sl], e[sl] = w2, e2
        assert int(N(cnt)[i]) == nb
        off += s
    assert bits_equal(N(tw), w) and bits_equal(N(te), e)


def test_fault_threshold_bit_exact(device, oracle_mod):
    from rramsim import ops
    u = np.random.default_rng(2).random(100_003).astype(np.float32)
    t = T(u, device)
    ops.fault_threshold(t, 0.25, 0.75)
    assert bits_equal(N(t), oracle_mod.fault_threshold(u, 0.25, 0.75))


def test_fault_init_vs_oracle(device, oracle_mod):
    import torch
    from rramsim import ops, split_thresholds
    n = 200_001
    tn, tz = split_thresholds(10, 20, 10)
    e = torch.empty(n, device=device)
    v = torch.empty(n, device=device)
    ops.fault_init(e, v, 5e6, 1e6, tn, tz, seed=1701, map_id=0, layer_id=2)
    e_ref, v_ref = oracle_mod.fault_init(n, 5e6, 1e6, tn, tz, 1701, 0, 2)
    assert bits_equal(N(v), v_ref)                    # integer RNG decisions: exact
    np.testing.assert_allclose(N(e), e_ref, rtol=2e-6, atol=2.0)  # logf/sincosf ulps


# -------------------------------------------------------------- injection
def _cfg_pair(p, **kw):
    from rramsim import make_inject_cfg
    c = make_inject_cfg(p, **kw)
    import oracle
    oc = oracle.InjectCfg(c.thr_fault, c.thr_neg, c.thr_zero, c.thr_sa1, c.stuck_scale, c.g_max,
                          c.quant_levels, c.var_sigma, c.cell_mode, 0)
    return c, oc


@pytest.mark.parametrize("n", [0, 1, 2, 7, 4096, 100_003, 4096 * 1000 + 3])
@pytest.mark.parametrize("mode", ["stuck", "quant", "stuck_scaled"])
def test_inject_bit_exact_vs_oracle(device, oracle_mod, n, mode):
    import torch
    from rramsim import ops
    kw = {"stuck": {}, "quant": dict(quant_levels=32, g_max=0.08),
          "stuck_scaled": dict(stuck_scale=0.05)}[mode]
    c, oc = _cfg_pair(0.05, neg=5, zero=90, pos=5, **kw)
    src = (np.random.default_rng(n).standard_normal(n) * 0.02).astype(np.float32)
    ts = T(src, device)
    out = torch.empty_like(ts)
    cnt = ops.counters(1, device)
    ops.inject(ts, out, c, seed=1701, map_id=3, layer_id=5, counter=cnt)
    ref, nb = oracle_mod.inject(src, oc, 1701, 3, 5)
    assert bits_equal(N(out), ref)
    assert int(N(cnt)[0]) == nb


def test_inject_beyond_2e31_elements(device, oracle_mod):
    """Maximum size: one blob of 2^31 + 4099 weights (8.6 GB in, 8.6 GB out;
    int64 element addressing past 2^31).  Windows at the start, across the
    2^31 boundary and at the ragged tail are checked element by element
    against the oracle's Philox stream and stuck-at rule (oracle.c draw /
    stuck_value), the broken count against the 3.8-sigma binomial bound
    (test_random_number_generator.cpp:17-19)."""
    import math
    import torch
    from rramsim import ops
    n = (1 << 31) + 4099
    p = 0.01
    c, _ = _cfg_pair(p, neg=10, zero=20, pos=10)
    src = torch.randn(n, device=device)
    out = torch.empty_like(src)
    cnt = ops.counters(1, device)
    seed, map_id, layer_id = 1701, 5, 3
    ops.inject(src, out, c, seed=seed, map_id=map_id, layer_id=layer_id, counter=cnt)
    torch.cuda.synchronize()
    for lo in (0, (1 << 31) - 1000, n - 1003):
        hi = min(n, lo + 1003)
        s_w = N(src[lo:hi])
        o_w = N(out[lo:hi])
        for i in range(lo, hi):
            pr = i >> 1
            r = oracle_mod.philox([pr & 0xFFFFFFFF, pr >> 32, map_id, (layer_id << 4) | 0],
                                  [seed & 0xFFFFFFFF, seed >> 32])
            rf, rv = (r[2], r[3]) if i & 1 else (r[0], r[1])
            if rf < c.thr_fault:
                want = np.float32(-1.0 if rv < c.thr_neg else (0.0 if rv < c.thr_zero else 1.0))
            else:
                want = s_w[i - lo]
            assert np.float32(o_w[i - lo]).view(np.uint32) == np.float32(want).view(np.uint32), i
    nb = int(N(cnt)[0])
    q = c.thr_fault / 2.0 ** 32
    assert abs(nb - n * q) <= 3.8 * math.sqrt(n * q * (1 - q)), (nb, n * q)
    del src, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("mode", ["var", "quant_var", "pair", "pair_quant_var"])
def test_inject_extensions_vs_oracle(device, oracle_mod, mode):
    import torch
    from rramsim import ops
    kw = {"var": dict(var_sigma=0.1), "quant_var": dict(quant_levels=16, g_max=0.1, var_sigma=0.05),
          "pair": dict(cell_mode=1, g_max=0.1, p_sa1=0.3),
          "pair_quant_var": dict(cell_mode=1, g_max=0.1, quant_levels=8, var_sigma=0.1)}[mode]
    c, oc = _cfg_pair(0.02, **kw)
    n = 65_537
    src = (np.random.default_rng(11).standard_normal(n) * 0.03).astype(np.float32)
    ts = T(src, device)
    out = torch.empty_like(ts)
    cnt = ops.counters(1, device)
    ops.inject(ts, out, c, seed=99, map_id=1, layer_id=0, counter=cnt)
    ref, nb = oracle_mod.inject(src, oc, 99, 1, 0)
    assert int(N(cnt)[0]) == nb                         # decisions are integer-exact
    np.testing.assert_allclose(N(out), ref, rtol=1e-5, atol=1e-7)  # expf/logf ulps


def test_inject_batched_alexnet_sizes_binomial(device):
    """Full AlexNet IP sizes (fc6/fc7/fc8 + biases, 58,631,144 weights): the
    broken fraction of each blob inside the 3.8-sigma binomial CI
    (test_random_number_generator.cpp:17-19 pattern), untouched weights
    unchanged, stuck values in {-1, 0, +1}."""
    import torch
    from rramsim import ops, make_inject_cfg
    shapes = [(4096, 9216), (4096,), (4096, 4096), (4096,), (1000, 4096), (1000,)]
    p = 0.01
    c = make_inject_cfg(p, 10, 20, 10)
    segs, srcs, outs = [], [], []
    g = torch.Generator(device=device).manual_seed(0)
    for i, sh in enumerate(shapes):
        s = torch.rand(sh, device=device, generator=g) * 0.5 + 2.0   # never in {-1,0,1}
        o = torch.empty_like(s)
        srcs.append(s)
        outs.append(o)
        segs.append((s, o, i, c))
    cnt = ops.counters(len(shapes), device)
    ops.inject_batched(segs, seed=1701, map_id=42, counters_t=cnt)
    torch.cuda.synchronize()
    counts = cnt.cpu().numpy()
    for i, (s, o) in enumerate(zip(srcs, outs)):
        changed = (o != s)
        nb = int(changed.sum())
        assert nb == counts[i]
        n = s.numel()
        assert abs(nb / n - p) <= 3.8 * math.sqrt(p * (1 - p) / n) + 1.0 / n
        vals = o[changed]
        assert bool(((vals == -1) | (vals == 0) | (vals == 1)).all())
    # -1/0/+1 split over all broken cells: 1/4, 1/2, 1/4
    allv = torch.cat([o[o != s] for s, o in zip(srcs, outs)])
    for val, q in ((-1, 0.25), (0, 0.5), (1, 0.25)):
        frac = float((allv == val).float().mean())
        assert abs(frac - q) <= 3.8 * math.sqrt(q * (1 - q) / allv.numel())


def test_inject_maps_independent_and_deterministic(device):
    import torch
    from rramsim import ops, make_inject_cfg
    c = make_inject_cfg(0.1)
    s = torch.full((1 << 20,), 5.0, device=device)
    a, b, a2 = torch.empty_like(s), torch.empty_like(s), torch.empty_like(s)
    ops.inject(s, a, c, 1, 0, 0)
    ops.inject(s, b, c, 1, 1, 0)
    ops.inject(s, a2, c, 1, 0, 0)
    torch.cuda.synchronize()
    assert torch.equal(a, a2)
    ma, mb = (a != 5), (b != 5)
    both = float((ma & mb).float().mean())
    assert abs(both - 0.01) < 0.002      # independent maps: P(both) = p^2


# -------------------------------------------------- threshold / SGD / fused
def test_threshold_strategy_bit_exact(device, oracle_mod):
    from rramsim import ops
    dw = (np.random.default_rng(4).standard_normal(300_001) * 1e-3).astype(np.float32)
    t = T(dw, device)
    cnt = ops.counters(1, device)
    ops.threshold_strategy(t, 5e-4, cnt)
    ref, n = oracle_mod.threshold(dw, 5e-4)
    assert bits_equal(N(t), ref) and int(N(cnt)[0]) == n


def test_sgd_update_and_fused_tail(device, oracle_mod):
    """SGDUpdate (sgd_solver.cu:6-12 with the CPU path's separate products,
    sgd_solver.cpp:222-228) and the fused Regularize + SGDUpdate + threshold +
    Update + Fail tail are bit-exact against the oracle's plain IEEE sequence
    (no FMA contraction on either side), including |update| exactly at the
    threshold and exactly at eps = 1e-20."""
    from rramsim import ops
    rng = np.random.default_rng(8)
    n = 100_003
    w, g, h = (rng.standard_normal(n).astype(np.float32) for _ in range(3))
    e = rng.normal(150, 100, n).astype(np.float32)
    e[:64] = 100.0                                    # exactly-zero crossings
    v = rng.integers(-1, 2, n).astype(np.float32)
    # boundary cells: zero history and decay so the update is exactly lr*g
    lr, thr = np.float32(0.01), np.float32(1e-3)
    h[:16] = 0.0
    g[:8] = thr / lr                                  # |update| ~ thr (ties resolved by rounding)
    g[8:16] = np.float32(1e-20) / lr
    tg, th = T(g, device), T(h, device)
    ops.sgd_update(tg, th, 0.9, 0.01)
    g2, h2 = oracle_mod.sgd_update(g, h, 0.9, 0.01)
    assert bits_equal(N(tg), g2) and bits_equal(N(th), h2)
    for decay in (0.0, 0.004):
        tw, tg, th, te = T(w, device), T(g, device), T(h, device), T(e, device)
        cnt = ops.counters(1, device)
        ops.fused_update_fail(tw, tg, th, te, T(v, device), decay, 0.9, 0.01, True, 1e-3, counter=cnt)
        w3, g3, h3, e3, nb = oracle_mod.fused_update_fail(w, g, h, e, v, decay, 0.9, 0.01, True, 1e-3)
        assert bits_equal(N(tw), w3) and bits_equal(N(tg), g3) and bits_equal(N(th), h3)
        assert bits_equal(N(te), e3) and int(N(cnt)[0]) == nb
        # the unfused kernels in the reference order give the same bits
        uw, ug, uh, ue = T(w, device), T(g, device), T(h, device), T(e, device)
        if decay:
            ops.axpy(decay, uw, ug)
        ops.sgd_update(ug, uh, 0.9, 0.01)
        ops.threshold_strategy(ug, 1e-3)
        ops.axpy(-1.0, ug, uw)
        c2 = ops.counters(1, device)
        ops.fail_apply(ug, uw, ue, T(v, device), counter=c2)
        assert bits_equal(N(uw), w3) and bits_equal(N(ue), e3) and int(N(c2)[0]) == nb


def test_fused_tail_batched_equals_per_blob(device, oracle_mod):
    """rram_fused_update_fail_batched (the solver's one-launch tail) gives the
    bits of one rram_fused_update_fail per blob and of the oracle: ragged
    sizes (incl. 1 and a non-multiple of the block chunk), a blob with no
    fault state, per-blob decay / lr / threshold, two segments sharing one
    broken counter."""
    from rramsim import ops
    rng = np.random.default_rng(21)
    sizes = [1, 4095, 2048, 300_001, 17, 96 * 363]
    blobs = []
    for k, n in enumerate(sizes):
        w, g, h = (rng.standard_normal(n).astype(np.float32) for _ in range(3))
        e = rng.normal(150, 100, n).astype(np.float32)
        v = rng.integers(-1, 2, n).astype(np.float32)
        faulty = k != 2
        blobs.append((w, g, h, e if faulty else None, v if faulty else None,
                      0.004 * (k % 2), np.float32(0.01 * (k + 1)), faulty, np.float32(1e-3 * (k + 1))))
    cnt_b = ops.counters(len(sizes), device)
    cnt_u = ops.counters(len(sizes), device)
    segs, outs_b, outs_u = [], [], []
    for k, (w, g, h, e, v, decay, lr, faulty, thr) in enumerate(blobs):
        tb = [T(x, device) if x is not None else None for x in (w, g, h, e, v)]
        tu = [T(x, device) if x is not None else None for x in (w, g, h, e, v)]
        slot = 0 if k in (0, 5) else k          # blobs 0 and 5 share counter 0
        segs.append((*tb, decay, lr, faulty, thr, cnt_b[slot:slot + 1] if faulty else None))
        ops.fused_update_fail(*tu, decay, 0.9, lr, faulty, thr,
                              counter=cnt_u[slot:slot + 1] if faulty else None)
        outs_b.append(tb)
        outs_u.append(tu)
    ops.fused_update_fail_batched(segs, 0.9)
    for k, (tb, tu) in enumerate(zip(outs_b, outs_u)):
        for a, b in zip(tb, tu):
            if a is not None:
                assert bits_equal(N(a), N(b)), k
        w, g, h, e, v, decay, lr, faulty, thr = blobs[k]
        if faulty:
            w3, g3, h3, e3, _ = oracle_mod.fused_update_fail(w, g, h, e, v, decay, 0.9, lr, True, thr)
            assert bits_equal(N(tb[0]), w3) and bits_equal(N(tb[3]), e3)
    assert (N(cnt_b) == N(cnt_u)).all()


# ------------------------------------------------------------------ GEMM
def test_gemm_kat_exact(device):
    import torch
    from rramsim import ops
    d = json.loads((GOLD / "gemm_kat.json").read_text())
    A, B, AT, BT = (T(np.array(d[k], np.float32), device) for k in ("A", "B", "A_T", "B_T"))
    ref = np.array(d["C"], np.float32).reshape(2, 4)
    for ta, tb, a, b in ((0, 0, A, B), (1, 0, AT, B), (1, 1, AT, BT), (0, 1, A, BT)):
        C = torch.full((2, 4), 7.0, device=device)
        ops.gemm(ta, tb, 2, 4, 3, 1.0, a, b, 0.0, C)
        assert np.array_equal(N(C), ref), (ta, tb)


def _gemm_ref(ta, tb, A, B):
    a = A.T if ta else A
    b = B.T if tb else B
    return a.astype(np.float64) @ b.astype(np.float64), np.abs(a).astype(np.float64) @ np.abs(b)


@pytest.mark.parametrize("shape", [(1, 1, 1), (31, 33, 17), (128, 128, 16), (200, 300, 1000),
                                   (256, 1000, 4096), (96, 3025, 363), (7, 5000, 3)])
@pytest.mark.parametrize("tt", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_random_vs_fp64(device, shape, tt):
    import torch
    from rramsim import ops
    M, Nn, K = shape
    ta, tb = tt
    rng = np.random.default_rng(M * 7 + Nn + K)
    A = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    B = rng.standard_normal((Nn, K) if tb else (K, Nn)).astype(np.float32)
    C0 = rng.standard_normal((M, Nn)).astype(np.float32)
    tc = T(C0, device)
    ops.gemm(ta, tb, M, Nn, K, 0.5, T(A, device), T(B, device), 1.5, tc)
    ref, scale = _gemm_ref(ta, tb, A, B)
    ref = 0.5 * ref + 1.5 * C0
    err = np.abs(N(tc) - ref)
    assert np.all(err <= 1e-5 * (0.5 * scale + 1.5 * np.abs(C0)) + 1e-6)   # fp32, 1e-5 of sum|a*b|


def test_gemm_epilogue_and_splitk(device):
    import torch
    from rramsim import ops
    rng = np.random.default_rng(17)
    M, Nn, K = 256, 1000, 4096          # AlexNet fc8 shape: split-K path
    X = rng.standard_normal((M, K)).astype(np.float32)
    W = rng.standard_normal((Nn, K)).astype(np.float32) * 0.01
    b = rng.standard_normal(Nn).astype(np.float32)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=device)
    out = torch.empty(M, Nn, device=device)
    ops.gemm_ex(0, 1, M, Nn, K, 1.0, T(X, device), K, T(W, device), K, 0.0, out, Nn,
                T(b, device), 2, True, ws)
    ref = np.maximum(X.astype(np.float64) @ W.T.astype(np.float64) + b, 0)
    scale = np.abs(X) @ np.abs(W.T) + np.abs(b)
    assert np.all(np.abs(N(out) - ref) <= 1e-5 * scale + 1e-6)
    out2 = torch.empty(M, Nn, device=device)
    ops.ip_fwd(T(X, device), T(W, device), T(b, device), out2, M, Nn, K, relu=True)
    assert np.all(np.abs(N(out2) - ref) <= 1e-5 * scale + 1e-6)


# ------------------------------------------------------------------ conv
CONV_CASES = [
    dict(x=(2, 3, 6, 4), cout=4, k=3, s=2, p=0, d=1, g=1),
    dict(x=(2, 3, 6, 4), cout=3, k=3, s=2, p=0, d=1, g=3),
    dict(x=(2, 3, 6, 4), cout=4, k=1, s=1, p=0, d=1, g=1),
    dict(x=(2, 3, 8, 7), cout=4, k=3, s=1, p=0, d=2, g=1),
    dict(x=(2, 3, 227, 227), cout=96, k=11, s=4, p=0, d=1, g=1),   # AlexNet conv1, 2 images
    dict(x=(2, 96, 27, 27), cout=256, k=5, s=1, p=2, d=1, g=2),    # conv2
    dict(x=(2, 256, 13, 13), cout=384, k=3, s=1, p=1, d=1, g=1),   # conv3
    dict(x=(3, 384, 13, 13), cout=384, k=3, s=1, p=1, d=1, g=2),   # conv4
    dict(x=(4, 32, 16, 16), cout=32, k=5, s=1, p=2, d=1, g=1),     # CIFAR conv2
    dict(x=(5, 480, 14, 14), cout=64, k=1, s=1, p=0, d=1, g=1),    # GoogLeNet 1x1
    dict(x=(2, 3, 40, 37), cout=64, k=7, s=2, p=3, d=1, g=1),      # GoogLeNet conv1 (64-bit tap mask)
    dict(x=(2, 5, 19, 23), cout=8, k=9, s=1, p=4, d=1, g=1),       # 81 taps, padded: the stepped gather
    dict(x=(2, 4, 21, 21), cout=6, k=5, s=2, p=3, d=2, g=2),       # dilation + groups + padding
]


@pytest.mark.parametrize("cs", CONV_CASES)
def test_conv_fwd_vs_oracle(device, oracle_mod, cs):
    import torch
    from rramsim import ops
    rng = np.random.default_rng(1701)
    x = rng.standard_normal(cs["x"]).astype(np.float32)
    w = (rng.standard_normal((cs["cout"], cs["x"][1] // cs["g"], cs["k"], cs["k"])) * 0.1).astype(np.float32)
    b = rng.standard_normal(cs["cout"]).astype(np.float32)
    d = ops.conv_desc(cs["x"], cs["cout"], cs["k"], cs["s"], cs["p"], cs["d"], cs["g"])
    y = torch.empty((cs["x"][0], cs["cout"], d.out_h, d.out_w), device=device)
    ops.conv2d_fwd(d, T(x, device), T(w, device), T(b, device), y)
    if np.prod(cs["x"]) * cs["cout"] * cs["k"] ** 2 < 5e7:
        ref = oracle_mod.conv_naive(x, w, b, cs["s"], cs["p"], cs["d"], cs["g"])
    else:
        ref = oracle_mod.conv_im2col(x, w, b, cs["s"], cs["p"], cs["d"], cs["g"])
    np.testing.assert_allclose(N(y), ref, atol=1e-4, rtol=1e-4)   # test_convolution_layer.cpp:256
    # fused ReLU epilogue
    ops.conv2d_fwd(d, T(x, device), T(w, device), T(b, device), y, relu=True)
    np.testing.assert_allclose(N(y), np.maximum(ref, 0), atol=1e-4, rtol=1e-4)


# Shapes aimed at the LDS-patch convolution (k_conv_patch: stride 1, 3x3 / 5x5,
# >= 128 output positions per image): 192-row weight tiles, 128-position tiles
# spanning two images, wide rows (56 x 56: 6 patch pieces per wave), padded M
# tiles, no padding, groups; and shapes it must leave to the im2col GEMM.
PATCH_CASES = [
    dict(x=(3, 8, 13, 13), cout=192, k=3, p=1, g=1),    # M = 192 tile, 169-position images
    dict(x=(2, 4, 56, 56), cout=128, k=3, p=1, g=1),    # wide rows
    dict(x=(2, 12, 28, 28), cout=224, k=5, p=2, g=1),   # 5x5, M padded to 256
    dict(x=(5, 8, 10, 13), cout=256, k=3, p=1, g=2),    # 130 positions: most tiles span two images
    dict(x=(2, 4, 20, 20), cout=128, k=5, p=0, g=1),    # 5x5 without padding (16 x 16 out)
    dict(x=(3, 32, 13, 13), cout=192, k=3, p=1, g=1),   # 16 | C: streamed x6 kernel, 96-row tiles, 2 super-tiles
    dict(x=(2, 16, 28, 28), cout=224, k=5, p=2, g=1),   # streamed 5x5, M padded to 256
    dict(x=(5, 32, 10, 13), cout=256, k=3, p=1, g=2),   # streamed, 130 positions: tiles over three images
    dict(x=(2, 16, 20, 20), cout=128, k=5, p=0, g=1),   # streamed 5x5 without padding
    dict(x=(3, 48, 27, 27), cout=256, k=5, p=2, g=2),   # AlexNet conv2 per-group shape: channel-octet x6 kernel, 128 x 256 tiles
    dict(x=(2, 32, 13, 13), cout=96, k=3, p=1, g=1),    # octet kernel: 96 of 128 rows (row masking), tiles over 2-3 images
    dict(x=(5, 16, 10, 13), cout=64, k=5, p=2, g=1),    # octet kernel: 5x5, 17-wide padded rows, 130 positions per image
    dict(x=(3, 64, 13, 13), cout=192, k=3, p=1, g=2),   # octet kernel: 64-row tiles (M = 96 per group), 4 K-tiles
    dict(x=(5, 32, 7, 7), cout=64, k=3, p=1, g=1),      # 49-position planes: whole-image tiles (2 per tile, last one short)
    dict(x=(3, 32, 7, 7), cout=128, k=5, p=2, g=1),     # 5x5 whole-image tiles, 128 x 128
    dict(x=(4, 48, 6, 7), cout=96, k=3, p=1, g=1),      # 42 positions: 3 images per tile
    dict(x=(3, 64, 7, 7), cout=192, k=3, p=1, g=2),     # whole-image tiles with groups
    dict(x=(7, 32, 5, 5), cout=64, k=3, p=1, g=1),      # 25 positions: capped at 3 images per tile
    dict(x=(4, 32, 4, 8), cout=64, k=3, p=0, g=1),      # 12 positions per image (2 x 6), no padding
    dict(x=(2, 6, 13, 13), cout=128, k=3, p=1, g=1),    # C % 4 != 0: im2col path
    dict(x=(2, 8, 12, 12), cout=128, k=3, p=0, g=1),    # 100 positions per image: im2col path
]


@pytest.fixture(params=["f32", "bf16x6"])
def conv_engine(request):
    """Runs a test under each matrix-core engine of the convolution forward
    (rram_set_f32_engine) and restores the previous one."""
    from rramsim import ops
    eng = ops.ENGINE_F32 if request.param == "f32" else ops.ENGINE_BF16X6
    prev = ops.set_f32_engine(eng)
    yield request.param
    ops.set_f32_engine(prev)


@pytest.mark.parametrize("cs", PATCH_CASES)
def test_conv_patch_shapes_vs_fp64(device, cs, conv_engine):
    """Forward convolution at the patch kernels' edges within 1e-4 of
    Σ|a·b| of a float64 reference (north_star tolerance, scale-aware), plain
    and with the fused ReLU, on both engines (fp32 MFMA and the bf16x6 split)."""
    import torch
    from rramsim import ops
    from _ref64 import check_conv
    rng = np.random.default_rng(99)
    x = rng.standard_normal(cs["x"]).astype(np.float32)
    w = (rng.standard_normal((cs["cout"], cs["x"][1] // cs["g"], cs["k"], cs["k"])) * 0.1).astype(np.float32)
    b = rng.standard_normal(cs["cout"]).astype(np.float32)
    d = ops.conv_desc(cs["x"], cs["cout"], cs["k"], 1, cs["p"], 1, cs["g"])
    y = torch.empty((cs["x"][0], cs["cout"], d.out_h, d.out_w), device=device)
    for relu in (False, True):
        ops.conv2d_fwd(d, T(x, device), T(w, device), T(b, device), y, relu=relu)
        torch.cuda.synchronize()
        check_conv(N(y), x, w, b, 1, cs["p"], cs["g"], relu=relu, what=f"conv {cs} relu={relu} {conv_engine}")


# AlexNet conv2 / conv3 / conv4 / conv5 at 4 images (Caffe-filler-like weight scale)
ENGINE_CASES = [
    dict(x=(2, 3, 227, 227), cout=96, k=11, p=0, g=1, s=4),    # conv1 (k_conv1_ring_x6)
    dict(x=(4, 96, 27, 27), cout=256, k=5, p=2, g=2),
    dict(x=(4, 256, 13, 13), cout=384, k=3, p=1, g=1),
    dict(x=(4, 384, 13, 13), cout=384, k=3, p=1, g=2),
    dict(x=(4, 384, 13, 13), cout=256, k=3, p=1, g=2),
    dict(x=(3, 64, 56, 56), cout=192, k=3, p=1, g=1),      # GoogLeNet conv2: row-aligned 64 x 128 tiles, 112 positions (28 per image)
    dict(x=(3, 128, 28, 28), cout=192, k=3, p=1, g=1),     # inception_3b/3x3: 64 x 256 contiguous tiles
    dict(x=(2, 3, 224, 224), cout=64, k=7, p=3, g=1, s=2),  # GoogLeNet conv1 (k_conv_s2_x6)
    dict(x=(6, 192, 7, 7), cout=384, k=3, p=1, g=1),       # inception_5b/3x3: whole-image tiles
]


@pytest.mark.parametrize("cs", ENGINE_CASES)
def test_conv_engine_bf16x6_accuracy_vs_f32(device, cs):
    """The bf16x6 engine is fp32-accurate, not reduced precision: against a
    float64 evaluation its error (in units of Σ|a·b|) is of the same size as
    the fp32-MFMA engine's, far inside the 1e-4 bound.  Prints both."""
    import torch
    from rramsim import ops
    from _ref64 import conv64
    rng = np.random.default_rng(7)
    x = np.maximum(rng.standard_normal(cs["x"]), 0).astype(np.float32)   # post-ReLU activations
    w = (rng.standard_normal((cs["cout"], cs["x"][1] // cs["g"], cs["k"], cs["k"])) * 0.01).astype(np.float32)
    b = rng.standard_normal(cs["cout"]).astype(np.float32)
    st = cs.get("s", 1)
    d = ops.conv_desc(cs["x"], cs["cout"], cs["k"], st, cs["p"], 1, cs["g"])
    ref, scale = conv64(x, w, b, st, cs["p"], cs["g"])
    err = {}
    prev = ops.get_f32_engine()
    try:
        for eng in (ops.ENGINE_F32, ops.ENGINE_BF16X6):
            ops.set_f32_engine(eng)
            assert ops.f32_engine_for_conv(d) == eng      # the shape really runs on that engine
            y = torch.empty((cs["x"][0], cs["cout"], d.out_h, d.out_w), device=device)
            ops.conv2d_fwd(d, T(x, device), T(w, device), T(b, device), y)
            torch.cuda.synchronize()
            r = np.abs(N(y).astype(np.float64) - ref) / scale
            err[eng] = (float(r.max()), float(r.mean()))
    finally:
        ops.set_f32_engine(prev)
    f32, x6 = err[ops.ENGINE_F32], err[ops.ENGINE_BF16X6]
    print(f"{cs}: max/mean err / Σ|a·b|: f32 {f32[0]:.2e}/{f32[1]:.2e}  bf16x6 {x6[0]:.2e}/{x6[1]:.2e}")
    assert x6[0] < 1e-6 and f32[0] < 1e-6          # fp32 level (the test bound is 1e-4)
    assert x6[0] <= 2.0 * f32[0] and x6[1] <= 2.0 * f32[1]


# Shapes of k_conv_s2_x6 (3 channels, 7 x 7, stride 2, <= 64 filters, >= 85
# output columns): GoogLeNet conv1, 40 of 64 filter rows with 4-row tiles,
# no padding with a partial last tile, 17 filters at padding 2
S2_CASES = [
    dict(x=(2, 3, 224, 224), cout=64, p=3),
    dict(x=(3, 3, 175, 173), cout=40, p=1),
    dict(x=(2, 3, 181, 180), cout=64, p=0),
    dict(x=(2, 3, 190, 191), cout=17, p=2),
]


@pytest.mark.parametrize("cs", S2_CASES)
def test_conv_s2_x6_vs_fp64(device, cs):
    """k_conv_s2_x6 within 1e-4 of Σ|a·b| of a float64 convolution, plain and
    with the fused ReLU; the output starts as NaN so every element is written."""
    import torch
    from rramsim import ops
    from _ref64 import check_conv
    rng = np.random.default_rng(23)
    x = rng.standard_normal(cs["x"]).astype(np.float32)
    w = (rng.standard_normal((cs["cout"], 3, 7, 7)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cs["cout"]).astype(np.float32)
    d = ops.conv_desc(cs["x"], cs["cout"], 7, 2, cs["p"], 1, 1)
    assert ops.f32_engine_for_conv(d) == ops.ENGINE_BF16X6
    for relu in (False, True):
        y = torch.full((cs["x"][0], cs["cout"], d.out_h, d.out_w), float("nan"), device=device)
        ops.conv2d_fwd(d, T(x, device), T(w, device), T(b, device), y, relu=relu)
        torch.cuda.synchronize()
        check_conv(N(y), x, w, b, 2, cs["p"], 1, relu=relu, what=f"conv s2 {cs} relu={relu}")


@pytest.mark.parametrize("cs", [CONV_CASES[0], CONV_CASES[1], CONV_CASES[4], CONV_CASES[12]])
def test_conv_fwd_unaligned_weights_nan_tail(device, oracle_mod, cs):
    """K % 4 != 0 (the unaligned 16-byte weight loader): the weights sit at a
    4-byte (not 16-byte) offset inside a NaN-filled buffer, so a float4 that
    runs past a row / group / the tensor end reads NaN; those lanes must be
    zeroed, and the last row's valid elements must survive the range check."""
    import torch
    from rramsim import ops
    rng = np.random.default_rng(7)
    x = rng.standard_normal(cs["x"]).astype(np.float32)
    w = (rng.standard_normal((cs["cout"], cs["x"][1] // cs["g"], cs["k"], cs["k"])) * 0.1).astype(np.float32)
    b = rng.standard_normal(cs["cout"]).astype(np.float32)
    d = ops.conv_desc(cs["x"], cs["cout"], cs["k"], cs["s"], cs["p"], cs["d"], cs["g"])
    big = torch.full((w.size + 9,), float("nan"), device=device)
    big[1:1 + w.size] = T(w.ravel(), device)
    wv = big[1:1 + w.size].view(w.shape)
    y = torch.empty((cs["x"][0], cs["cout"], d.out_h, d.out_w), device=device)
    ops.conv2d_fwd(d, T(x, device), wv, T(b, device), y)
    if np.prod(cs["x"]) * cs["cout"] * cs["k"] ** 2 < 5e7:
        ref = oracle_mod.conv_naive(x, w, b, cs["s"], cs["p"], cs["d"], cs["g"])
    else:
        ref = oracle_mod.conv_im2col(x, w, b, cs["s"], cs["p"], cs["d"], cs["g"])
    np.testing.assert_allclose(N(y), ref, atol=1e-4, rtol=1e-4)


def _bwd_ref64(fwd, inputs, dy):
    """float64 gradients of fwd(*inputs) for upstream dy, and their error scale:
    the same backward evaluated on |inputs| and |dy| (= Σ|a·b| of each gradient
    contraction, test_convolution_layer.cpp:256 tolerance made scale-aware)."""
    import torch
    xs = [t.double().clone().requires_grad_(True) for t in inputs]
    fwd(*xs).backward(dy.double())
    xa = [t.double().abs().clone().requires_grad_(True) for t in inputs]
    fwd(*xa).backward(dy.double().abs())
    return [t.grad.numpy() for t in xs], [t.grad.numpy() for t in xa]


@pytest.mark.parametrize("cs", CONV_CASES[:4] + [CONV_CASES[8], CONV_CASES[6], CONV_CASES[12]])
def test_conv_bwd_vs_fp64(device, cs):
    """Convolution backward (conv_layer.cu:26-56: weight GEMM accumulate, bias
    sum, data GEMM + col2im) within 1e-4 of Σ|a·b| of a float64 reference."""
    import torch
    from rramsim import ops
    torch.manual_seed(0)
    x = torch.randn(cs["x"], dtype=torch.float32)
    w = torch.randn(cs["cout"], cs["x"][1] // cs["g"], cs["k"], cs["k"]) * 0.1
    b = torch.randn(cs["cout"])
    fwd = lambda xx, ww, bb: torch.nn.functional.conv2d(xx, ww, bb, cs["s"], cs["p"], cs["d"], cs["g"])  # noqa: E731
    dy = torch.randn_like(fwd(x, w, b))
    (gx, gw, gb), (sx, sw, sb) = _bwd_ref64(fwd, (x, w, b), dy)
    d = ops.conv_desc(cs["x"], cs["cout"], cs["k"], cs["s"], cs["p"], cs["d"], cs["g"])
    dw = torch.zeros_like(w, device=device)
    db = torch.zeros_like(b, device=device)
    dx = torch.empty_like(x, device=device)
    ws = torch.empty(ops.conv2d_bwd_workspace(d, 2) // 4 + 1, device=device)   # forces chunking
    ops.conv2d_bwd(d, x.to(device), w.to(device), dy.to(device), dw, db, dx, ws)
    torch.cuda.synchronize()
    import _ref64 as R
    for got, ref, sc, nm in ((dw, gw, sw, "dW"), (db, gb, sb, "db"), (dx, gx, sx, "dX")):
        R.assert_scaled(got.cpu().numpy(), ref, sc, nm)


DX_FWD_CASES = [  # fwd: the flipped-kernel forward runs (>= 128 tiles of 32 channels x 128 positions)
    dict(x=(64, 32, 16, 16), cout=32, k=5, s=1, p=2, d=1, g=1, fwd=True),     # CIFAR conv2
    dict(x=(6, 96, 27, 27), cout=256, k=5, s=1, p=2, d=1, g=2, fwd=True),     # AlexNet conv2, groups
    dict(x=(8, 384, 13, 13), cout=384, k=3, s=1, p=1, d=1, g=2, fwd=True),    # conv4
    dict(x=(6, 480, 14, 14), cout=64, k=1, s=1, p=0, d=1, g=1, fwd=True),     # GoogLeNet 1x1
    dict(x=(40, 5, 19, 23), cout=8, k=9, s=1, p=4, d=1, g=1, fwd=True),       # 81 taps
    dict(x=(58, 4, 13, 11), cout=6, k=3, s=1, p=2, d=2, g=2, fwd=True),       # dilation + groups + padding
    dict(x=(300, 3, 8, 7), cout=4, k=3, s=1, p=0, d=2, g=1, fwd=True),        # flipped padding 4 > kernel
    dict(x=(230, 3, 9, 8), cout=5, k=(3, 1), s=1, p=(1, 0), d=1, g=1, fwd=True),  # non-square kernel
    dict(x=(4, 32, 8, 8), cout=64, k=5, s=1, p=2, d=1, g=1, fwd=False),       # small grid: GEMM + col2im
    dict(x=(2, 3, 6, 6), cout=4, k=3, s=1, p=3, d=1, g=1, fwd=False),         # pad > k-1: GEMM + col2im
]


@pytest.mark.parametrize("eng", ["f32", "bf16x6"])
@pytest.mark.parametrize("cs", DX_FWD_CASES)
def test_conv_bwd_dx_stride1_vs_fp64(device, cs, eng):
    """Stride-1 data gradient as a forward convolution of dY with the flipped,
    channel-transposed kernel (padding dil*(k-1) - pad) instead of the data GEMM
    + col2im (conv_layer.cu:47-52), on both fp32 engines, with and without the
    weight gradient in the same call.  Which path ran is observable: with dX
    alone the forward needs only the flipped kernel's bytes of workspace, the
    col2im path one image's column matrix."""
    import torch
    from rramsim import ops
    from rramsim import _kernels as Kmod
    kh, kw = cs["k"] if isinstance(cs["k"], tuple) else (cs["k"], cs["k"])
    ph, pw = cs["p"] if isinstance(cs["p"], tuple) else (cs["p"], cs["p"])
    torch.manual_seed(3)
    x = torch.randn(cs["x"], dtype=torch.float32)
    w = torch.randn(cs["cout"], cs["x"][1] // cs["g"], kh, kw) * 0.1
    b = torch.randn(cs["cout"])
    fwd = lambda xx, ww, bb: torch.nn.functional.conv2d(xx, ww, bb, 1, (ph, pw), cs["d"], cs["g"])  # noqa: E731
    dy = torch.randn_like(fwd(x, w, b))
    (gx, gw, gb), (sx, sw, sb) = _bwd_ref64(fwd, (x, w, b), dy)
    d = ops.conv_desc(cs["x"], cs["cout"], (kh, kw), 1, (ph, pw), cs["d"], cs["g"])
    import _ref64 as R
    wt_floats = w.numel()
    col_floats = cs["x"][1] * kh * kw * d.out_h * d.out_w
    xd, wd, dyd = x.to(device), w.to(device), dy.to(device)
    prev = ops.set_f32_engine(ops.ENGINE_F32 if eng == "f32" else ops.ENGINE_BF16X6)
    try:
        if wt_floats < col_floats:
            small = torch.empty(wt_floats, device=device)
            dx = torch.full_like(x, float("nan"), device=device)
            if cs["fwd"]:
                ops.conv2d_bwd(d, xd, wd, dyd, None, None, dx, small)
                torch.cuda.synchronize()
                R.assert_scaled(dx.cpu().numpy(), gx, sx, "dX (flipped-kernel forward)")
            else:
                with pytest.raises(Kmod.RramError):
                    ops.conv2d_bwd(d, xd, wd, dyd, None, None, dx, small)
        for with_dw in (False, True):
            dw = torch.zeros_like(w, device=device) if with_dw else None
            dx = torch.full_like(x, float("nan"), device=device)
            ws = torch.empty(ops.conv2d_bwd_workspace(d, cs["x"][0]) // 4 + 1, device=device)
            ops.conv2d_bwd(d, xd, wd, dyd, dw, None, dx, ws)
            torch.cuda.synchronize()
            R.assert_scaled(dx.cpu().numpy(), gx, sx, "dX")
            if with_dw:
                R.assert_scaled(dw.cpu().numpy(), gw, sw, "dW")
    finally:
        ops.set_f32_engine(prev)


def test_ip_bwd_vs_fp64(device):
    """InnerProduct backward (inner_product_layer.cu:40-75) at LeNet ip1 and
    AlexNet fc6 shapes within 1e-4 of Σ|a·b| of a float64 reference."""
    import torch
    import _ref64 as R
    from rramsim import ops
    torch.manual_seed(1)
    for M, Nn, K in ((64, 500, 800), (256, 4096, 9216)):
        x, w, b = torch.randn(M, K), torch.randn(Nn, K) * 0.05, torch.randn(Nn)
        fwd = lambda xx, ww, bb: xx @ ww.T + bb  # noqa: E731
        dy = torch.randn(M, Nn)
        (gx, gw, gb), (sx, sw, sb) = _bwd_ref64(fwd, (x, w, b), dy)
        dw = torch.zeros(Nn, K, device=device)
        db = torch.zeros(Nn, device=device)
        dx = torch.empty(M, K, device=device)
        ops.ip_bwd(x.to(device), w.to(device), dy.to(device), dw, db, dx, M, Nn, K)
        torch.cuda.synchronize()
        for got, ref, sc, nm in ((dw, gw, sw, "dW"), (db, gb, sb, "db"), (dx, gx, sx, "dX")):
            R.assert_scaled(got.cpu().numpy(), ref, sc, f"{nm} {M}x{Nn}x{K}")


def test_im2col_col2im_vs_oracle(device, oracle_mod):
    import torch
    from rramsim import ops
    im = np.random.default_rng(3).standard_normal((5, 15, 15)).astype(np.float32)
    ref = oracle_mod.im2col(im, 3, 3, 0, 0, 2, 2, 3, 3)           # test_im2col_kernel.cu:36-62
    col = torch.empty(ref.shape, device=device)
    ops.im2col(T(im, device), 5, 15, 15, 3, 3, 0, 0, 2, 2, 3, 3, col)
    assert bits_equal(N(col), ref)
    back = torch.empty((5, 15, 15), device=device)
    ops.col2im(col, 5, 15, 15, 3, 3, 0, 0, 2, 2, 3, 3, back)
    np.testing.assert_allclose(N(back), oracle_mod.col2im(ref, 5, 15, 15, 3, 3, 0, 0, 2, 2, 3, 3),
                               rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------- support layers
@pytest.mark.parametrize("outer,C,inner,ignore", [(100, 10, 1, -1), (7, 10, 5, 3), (64, 64, 1, -1), (1, 2, 1, -1),
                                                  (256, 1000, 1, -1), (50, 1000, 1, 7), (3, 100, 50, -1),
                                                  (20000, 100, 1, -1), (6, 1500, 2, 4)])
def test_accuracy_small_head_single_launch(device, oracle_mod, outer, C, inner, ignore):
    """Accuracy == the restated AccuracyLayer, with ties, an ignore label,
    spatial positions, and the ratio output (top-1 and top-3), twice per case:
    the one-block kernel (classes <= 64), the single-launch multi-block kernel
    (per-block slots + last-block sum; its ticket re-arms itself, so the
    second call must agree), and past 4096 blocks the atomics + ratio form;
    C = 1500 takes the strided-loop branch (class values batched up to 1024)."""
    import torch
    from rramsim import ops
    rng = np.random.default_rng(outer + C)
    x = rng.integers(-3, 4, (outer, C, inner)).astype(np.float32)   # many exact ties
    label = rng.integers(0, C, (outer, inner)).astype(np.float32)
    for k in (1, 3, 1):
        if k > C:
            continue
        cor, cnt, ratio = (torch.full((1,), -5.0, device=device) for _ in range(3))
        ops.accuracy(T(x, device), T(label, device), cor, cnt, outer, C, inner, top_k=k, ignore=ignore, ratio=ratio)
        hit = n = 0
        for o in range(outer):
            for q in range(inner):
                lv = int(label[o, q])
                if ignore >= 0 and lv == ignore:
                    continue
                col = x[o, :, q]
                rank = int(np.sum((col > col[lv]) | ((col == col[lv]) & (np.arange(C) > lv))))
                hit += rank < k
                n += 1
        assert int(N(cor)[0]) == hit and int(N(cnt)[0]) == n
        assert abs(float(N(ratio)[0]) - hit / max(n, 1)) < 1e-6


def test_pool_lrn_softmax_accuracy_vs_oracle(device, oracle_mod):
    import torch
    from rramsim import ops
    rng = np.random.default_rng(6)
    x = rng.standard_normal((3, 8, 13, 13)).astype(np.float32)
    for method, k, s, p in (("MAX", 3, 2, 0), ("AVE", 3, 2, 1), ("MAX", 2, 2, 0), ("AVE", 5, 3, 0)):
        ref = oracle_mod.pool(x, k, s, p, method)
        y = torch.empty(ref.shape, device=device)
        mask = torch.empty(ref.shape, dtype=torch.int32, device=device)
        geom = (3, 8, 13, 13, ref.shape[2], ref.shape[3], k, k, s, s, p, p)
        ops.pool_fwd(T(x, device), y, mask, geom, 0 if method == "MAX" else 1)
        np.testing.assert_allclose(N(y), ref, rtol=1e-6, atol=1e-6)
    ref = oracle_mod.lrn(x, 5, 1e-4, 0.75, 1.0)
    y = torch.empty_like(T(x, device))
    ops.lrn_fwd(T(x, device), y, None, 3, 8, 13, 13, 5, 1e-4, 0.75, 1.0)
    np.testing.assert_allclose(N(y), ref, rtol=1e-5, atol=1e-6)
    logits = rng.standard_normal((256, 1000)).astype(np.float32)
    pr = torch.empty(256, 1000, device=device)
    ops.softmax_fwd(T(logits, device), pr, 256, 1000, 1)
    np.testing.assert_allclose(N(pr), oracle_mod.softmax(logits), rtol=1e-5, atol=1e-7)
    label = rng.integers(0, 1000, 256).astype(np.float32)
    logits[:, 5] = logits[:, 7]                       # ties exercise the pair ordering
    cor, cnt = torch.zeros(1, device=device), torch.zeros(1, device=device)
    for k in (1, 5):
        ops.accuracy(T(logits, device), T(label, device), cor, cnt, 256, 1000, 1, top_k=k)
        assert int(N(cor)[0]) == oracle_mod.accuracy(logits, label, k) and int(N(cnt)[0]) == 256


IM2COL_CASES = [  # (C, H, W, kh, kw, ph, pw, sh, sw, dh, dw)
    (3, 32, 32, 5, 5, 2, 2, 1, 1, 1, 1),     # CIFAR conv1: Ho*Wo % 4 == 0 (16-byte stores)
    (32, 8, 8, 5, 5, 2, 2, 1, 1, 1, 1),      # CIFAR conv3
    (3, 227, 227, 11, 11, 0, 0, 4, 4, 1, 1), # AlexNet conv1: 55 x 55 (scalar form)
    (5, 9, 6, 3, 3, 1, 1, 1, 1, 1, 1),       # Wo = 6: quads wrap output rows
    (4, 5, 2, 3, 1, 1, 0, 1, 1, 1, 1),       # Wo = 2: a quad spans two rows
    (2, 11, 13, 3, 3, 2, 1, 2, 1, 2, 1),     # stride + dilation + padding
    (1, 1, 1, 1, 1, 0, 0, 1, 1, 1, 1),       # 1 x 1
]


@pytest.mark.parametrize("cs", IM2COL_CASES)
def test_im2col_col2im_bit_exact(device, oracle_mod, cs):
    """im2col (im2col.cu:9-36; the 4-position 16-byte-store form when Ho*Wo %
    4 == 0) bit-exact against the oracle; col2im (im2col.cu:65-116) against the
    oracle's accumulation within fp32 summation-order tolerance."""
    import torch
    from rramsim import ops
    C_, H, W, kh, kw, ph, pw, sh, sw, dh, dw = cs
    rng = np.random.default_rng(sum(cs))
    im = rng.standard_normal((C_, H, W)).astype(np.float32)
    ref = oracle_mod.im2col(im, kh, kw, ph, pw, sh, sw, dh, dw)
    col = torch.full(ref.shape, float("nan"), device=device)
    ops.im2col(T(im, device), C_, H, W, kh, kw, ph, pw, sh, sw, dh, dw, col)
    assert bits_equal(N(col), ref)
    back = torch.empty((C_, H, W), device=device)
    ops.col2im(T(ref, device), C_, H, W, kh, kw, ph, pw, sh, sw, dh, dw, back)
    np.testing.assert_allclose(N(back), oracle_mod.col2im(ref, C_, H, W, kh, kw, ph, pw, sh, sw, dh, dw),
                               rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("shape,cout,k,pad,relu", [
    ((100, 32, 16, 16), 32, 5, 2, True),    # CIFAR-10 quick / full conv2 (split-K forward)
    ((100, 32, 8, 8), 64, 5, 2, True),      # CIFAR-10 quick conv3
    ((100, 20, 12, 12), 50, 5, 0, False),   # LeNet conv2
    ((7, 33, 9, 9), 40, 3, 1, True),        # ragged: K % 32 != 0, N % 128 != 0
])
def test_conv_fwd_split_k_vs_fp64(device, shape, cout, k, pad, relu):
    """The fp32 convolution forward with K split over workgroups
    (conv_fwd_split: thin, short-grid layers) + k_splitk_reduce_nchw: within
    fp32 accumulation error of float64 (<= 2e-6 of sum|a*b| + |bias|), bias and
    ReLU applied once, NCHW layout."""
    import torch
    from rramsim import ops
    from _ref64 import conv64, assert_scaled
    rng = np.random.default_rng(5)
    x = rng.standard_normal(shape).astype(np.float32)
    w = (rng.standard_normal((cout, shape[1], k, k)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    d = ops.conv_desc(shape, cout, k, 1, pad)
    y = torch.full((shape[0], cout, d.out_h, d.out_w), float("nan"), device=device)
    ops.conv2d_fwd(d, T(x, device), T(w, device), T(b, device), y, relu=relu)
    ref, scale = conv64(x, w, b, 1, pad)
    assert_scaled(N(y), ref, scale, "conv fwd split-K", tol=2e-6, relu=relu)


@pytest.mark.parametrize("shape,cout,k,pad,chunk", [
    ((100, 3, 32, 32), 32, 5, 2, None),     # CIFAR-10 full conv1 (bias folded into the dW GEMM)
    ((100, 32, 16, 16), 32, 5, 2, None),    # conv2
    ((100, 32, 8, 8), 64, 5, 2, None),      # conv3
    ((9, 16, 8, 8), 24, 3, 1, 2),           # workspace for 2 images: chunks of 2 and a last one of 1
])
def test_conv_bwd_bias_folded_vs_fp64(device, shape, cout, k, pad, chunk):
    """The conv bias gradient as one more column of the split weight-gradient
    GEMM (a ones row after the im2col rows; k_splitk_reduce_dwdb routes it to
    db) accumulates into db like the separate reduction: db, dW and dX within
    1e-5 of sum|a*b| of float64, over several image chunks too."""
    import torch
    from rramsim import ops
    import _ref64 as R
    torch.manual_seed(3)
    x = torch.randn(shape)
    w = torch.randn(cout, shape[1], k, k) * 0.1
    b = torch.randn(cout)
    fwd = lambda xx, ww, bb: torch.nn.functional.conv2d(xx, ww, bb, 1, pad)  # noqa: E731
    dy = torch.randn_like(fwd(x, w, b))
    (gx, gw, gb), (sx, sw, sb) = _bwd_ref64(fwd, (x, w, b), dy)
    d = ops.conv_desc(shape, cout, k, 1, pad)
    dw = torch.full_like(w, 0.25, device=device)          # accumulates: += on 0.25 / -0.5
    db = torch.full_like(b, -0.5, device=device)
    dx = torch.empty_like(x, device=device)
    ws = torch.empty(ops.conv2d_bwd_workspace(d, chunk or shape[0]) // 4 + 64, device=device)
    ops.conv2d_bwd(d, x.to(device), w.to(device), dy.to(device), dw, db, dx, ws)
    torch.cuda.synchronize()
    R.assert_scaled(dw.cpu().numpy() - 0.25, gw, sw, "dW", tol=1e-5)
    R.assert_scaled(db.cpu().numpy() + 0.5, gb, sb, "db", tol=1e-5)
    R.assert_scaled(dx.cpu().numpy(), gx, sx, "dX", tol=1e-5)
