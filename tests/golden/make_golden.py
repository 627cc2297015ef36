"""Generate the known-answer fixtures in tests/golden/.

The reference ships no fault-injection tests and cannot be built
here (no protobuf/glog/boost/cblas — SURVEY.md §0.4), so these vectors are
hand-derived from the reference source with an independent numpy float32
restatement (NOT the C oracle), covering the edge cases SURVEY.md §8c lists:

  fail_apply  — GaussianFailureMaker::Fail_cpu / FailKernel
                (src/caffe/failure_maker.cpp:55-81, failure_maker.cu:23-41):
                e <= 0 at start (re-pin, Appendix A Q4), exact-zero crossings,
                |dw| at / just below / just above 1e-20, NaN dw, and fp32-inexact
                decrements at means 5e6 / 3.1e6 / 3e7 / 7e7 / 1e8 (Q1),
                after k in {1, 2, 5} Fail() calls.
  gemm        — test_util_blas.cpp:20-89 known answer (stored for completeness).
  threshold   — FailureThresholdKernel (failure_maker.cu:5-16) on chosen uniforms.

Run:  python tests/golden/make_golden.py   (writes *.json next to this file)
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

OUT = Path(__file__).resolve().parent
f32 = np.float32


def fail_step(dw, w, e, v, dec=f32(100.0), eps=f32(1e-20)):
    """One reference Fail() on float32 arrays (numpy restatement)."""
    w, e = w.copy(), e.copy()
    for j in range(len(w)):
        if e[j] <= f32(0):
            w[j] = v[j]
        else:
            if np.abs(dw[j]) < eps:
                continue
            e[j] = f32(e[j] - dec)
            if e[j] <= f32(0):
                w[j] = v[j]
    return w, e


def bits(a):
    return [int(x) for x in np.asarray(a, np.float32).view(np.uint32)]


def fail_cases():
    eps = f32(1e-20)
    below = np.nextafter(eps, f32(0))
    above = np.nextafter(eps, f32(1))
    e0 = np.array([0, -5, 100, 100.5, 200, 250, 1e8, 3.1e6, 3e7, 7e7, 5e6, 16777217.0,
                   300, 300, 300, 300, 300, 150, 1e-30, 99.99999], f32)
    v = np.array([-1, 0, 1, -1, 0, 1, -1, 0, 1, -1, 0, 1, -1, 0, 1, -1, 0, 1, -1, 0], f32)
    w0 = np.linspace(-0.7, 0.9, len(e0)).astype(f32)
    dws = [
        np.array([0.5, 0.0, 0.5, 0.5, -0.3, 1e-3, 0.1, 0.2, -0.2, 0.3, 1.0, 2.0,
                  eps, -eps, below, -below, above, np.nan, 0.25, 0.5], f32),
        np.array([0.0, 0.0, 0.0, 0.4, 0.4, 0.4, 0.4, 0.4, 0.4, 0.4, 0.4, 0.4,
                  eps, eps, eps, eps, eps, eps, eps, eps], f32),
        np.full(len(e0), 0.01, f32),
        np.array([1e-21] * 10 + [1.0] * 10, f32),
        np.array([np.inf, -np.inf] * 10, f32),
    ]
    cases = []
    for k in (1, 2, 5):
        w, e = w0.copy(), e0.copy()
        steps = []
        for i in range(k):
            dw = dws[i % len(dws)]
            w, e = fail_step(dw, w, e, v)
            steps.append({"dw_bits": bits(dw)})
        cases.append({"k": k, "e0_bits": bits(e0), "v_bits": bits(v), "w0_bits": bits(w0),
                      "steps": steps, "w_bits": bits(w), "e_bits": bits(e),
                      "broken": int(np.sum(e <= 0))})
    return cases


def main():
    (OUT / "fail_apply_kat.json").write_text(json.dumps(
        {"source": "numpy float32 restatement of failure_maker.cpp:55-81", "decrement": 100.0,
         "eps": 1e-20, "cases": fail_cases()}, indent=1))
    u = np.array([0.0, 0.2499, 0.25, 0.5, 0.7499999, 0.75, 0.99999994, 0.1, 0.9], f32)
    s1, s2 = f32(10 / 40), f32(30 / 40)
    thr = np.where(u < s1, f32(-1), np.where(u < s2, f32(0), f32(1))).astype(f32)
    (OUT / "threshold_kat.json").write_text(json.dumps(
        {"source": "failure_maker.cu:5-16 with default neg/zero/pos = 10/20/10",
         "split1": float(s1), "split2": float(s2), "u_bits": bits(u), "v_bits": bits(thr)},
        indent=1))
    (OUT / "gemm_kat.json").write_text(json.dumps(
        {"source": "src/caffe/test/test_util_blas.cpp:20-89",
         "A": [1, 2, 3, 4, 5, 6], "B": list(range(1, 13)),
         "A_T": [1, 4, 2, 5, 3, 6], "B_T": [1, 5, 9, 2, 6, 10, 3, 7, 11, 4, 8, 12],
         "C": [38, 44, 50, 56, 83, 98, 113, 128]}, indent=1))


if __name__ == "__main__":
    main()
