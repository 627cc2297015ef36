"""CPU check that the fp32-level guard of the bf16x6 engine can fail
(tests/test_gpu_fp32_guard.py, bounds in tests/_ref64.py x6_guard_failures).

A numpy model of the two engines' arithmetic on dot products of the bench's
contraction lengths (AlexNet conv1-5, fc6, fc7 at b256):
  * fp32 MFMA (v_mfma_f32_32x32x2_f32): exact products, fp32 accumulation
    after every 2-long K block;
  * bf16x6 (csrc/x6.hip x6::mfma6): each fp32 operand split exactly into
    three bf16 terms (round-to-nearest-even), the six products
    al·bh, ah·bl, am·bm, am·bh, ah·bm, ah·bh of each 16-long K block summed
    exactly and accumulated in fp32 in that order.
The full split passes the guard; leaving out any one of the five lower
product terms, or keeping only the bf16x3 form (am·bh, ah·bm, ah·bh), fails
it — every such variant also passes the 1e-4 · Σ|a·b| north_star gate, which
is why the guard exists.  No GPU: this pins the criterion, the GPU file pins
the kernels.
"""
import numpy as np
import pytest

from _ref64 import TOL, x6_guard_failures

# (name, K, activation scale, weight std) of the bench's contractions
LAYERS = [("conv1", 363, 128.0, 0.01), ("conv2", 1200, 3.0, 0.01), ("conv3", 2304, 1.0, 0.01),
          ("conv4", 1728, 1.0, 0.01), ("conv5", 1728, 1.0, 0.01), ("fc6", 9216, 1.0, 0.005),
          ("fc7", 4096, 1.0, 0.005)]
TERMS = ["al*bh", "ah*bl", "am*bm", "am*bh", "ah*bm", "ah*bh"]


def bf16(x):
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return (((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16).astype(np.uint32).view(np.float32)


def split3(x):
    h = bf16(x)
    r = (x - h).astype(np.float32)       # exact in fp32
    m = bf16(r)
    return h, m, bf16((r - m).astype(np.float32))


def fp32_acc(blocks):
    """blocks: list of [E] float64 exact block sums -> fp32 accumulation."""
    acc = np.zeros(blocks[0].shape, np.float32)
    for s in blocks:
        acc = (acc.astype(np.float64) + s).astype(np.float32)
    return acc


def engines(a, b, drop=()):
    K = a.shape[1]
    f32 = fp32_acc([(a[:, k:k + 2].astype(np.float64) * b[:, k:k + 2]).sum(1) for k in range(0, K, 2)])
    (ah, am, al), (bh, bm, bl) = split3(a), split3(b)
    ops = [(al, bh), (ah, bl), (am, bm), (am, bh), (ah, bm), (ah, bh)]
    blocks = []
    for k in range(0, K, 16):
        for t, (p, q) in enumerate(ops):
            if TERMS[t] not in drop:
                blocks.append((p[:, k:k + 16].astype(np.float64) * q[:, k:k + 16]).sum(1))
    return f32, fp32_acc(blocks)


def errors(a, b, drop=()):
    ref = (a.astype(np.float64) * b).sum(1)
    scale = np.abs(a.astype(np.float64) * b).sum(1)
    out = []
    for y in engines(a, b, drop):
        r = np.abs(y - ref) / scale
        out.append((float(r.max()), float(r.mean())))
    return out


def operands(K, act, std, seed, E=768):
    rng = np.random.default_rng(seed)
    a = (np.maximum(rng.standard_normal((E, K)), 0) * act).astype(np.float32)     # post-ReLU activations
    b = (rng.standard_normal((E, K)) * std).astype(np.float32)
    return a, b


@pytest.mark.parametrize("layer", LAYERS, ids=[x[0] for x in LAYERS])
def test_guard_passes_full_split_and_rejects_dropped_terms(layer):
    name, K, act, std = layer
    a, b = operands(K, act, std, seed=K)
    f32, x6 = errors(a, b)
    assert not x6_guard_failures(x6, f32), (name, x6, f32)
    variants = [(t,) for t in TERMS[:5]] + [("al*bh", "ah*bl", "am*bm")]      # single drops, bf16x3
    for drop in variants:
        f32d, x6d = errors(a, b, drop)
        assert f32d == f32
        assert x6d[0] <= TOL or drop[0] in ("am*bh", "ah*bm")   # the 2^-16 drops pass the 1e-4 gate
        assert x6_guard_failures(x6d, f32), f"{name}: dropping {drop} passed the guard ({x6d} vs fp32 {f32})"
