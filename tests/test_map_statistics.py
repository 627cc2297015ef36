"""The C2 line's per-map statistics (scripts/bench_workloads.py
map_statistics): mean, sample std and 95 % CI half-width from all-reduced
moments equal numpy's over the same per-map values, split over ranks as the
bench all-reduces them (CPU only)."""
import importlib.util
import pathlib

import numpy as np

_P = pathlib.Path(__file__).resolve().parents[1] / "scripts" / "bench_workloads.py"


def _mod():
    spec = importlib.util.spec_from_file_location("bench_workloads", _P)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_ci_half_width_matches_per_map_spread():
    m = _mod()
    rng = np.random.default_rng(5)
    acc = 0.1 + 0.02 * rng.standard_normal(1000)           # 1000 maps' accuracies
    ranks = np.array_split(acc, 8)                          # 8 ranks' timed maps
    s = sum(float(r.sum()) for r in ranks)
    s2 = sum(float((r * r).sum()) for r in ranks)
    st = m.map_statistics(s, s2, sum(len(r) for r in ranks))
    assert st["maps"] == 1000
    assert abs(st["mean"] - acc.mean()) < 1e-12
    assert abs(st["std"] - acc.std(ddof=1)) < 1e-9
    assert abs(st["ci95"] - 1.96 * acc.std(ddof=1) / np.sqrt(1000)) < 1e-10


def test_degenerate_cases():
    m = _mod()
    one = m.map_statistics(0.25, 0.0625, 1)
    assert one["mean"] == 0.25 and one["std"] == 0.0 and one["ci95"] == 0.0
    const = m.map_statistics(5 * 0.1, 5 * 0.01, 5)          # identical maps: rounding must not go negative
    assert const["std"] >= 0.0 and const["ci95"] < 1e-7
