"""Caffe CPU mode for any of the benchmark nets — TEST INFRASTRUCTURE ONLY
(bench.py's cpu_baseline leg and tests/ import it; the product never does).

A TEST-phase forward driven by the same prototxt the GPU net parses
(rramsim.models), layer by layer in the reference's CPU code paths:
  Convolution   per-image im2col_cpu + cblas_sgemm per group + the rank-1 bias
                sgemm (conv_layer.cpp:7-27 via caffe_cpu.c, cc_conv)
  InnerProduct  one sgemm + bias (inner_product_layer.cpp:63-82, cc_ip)
  ReLU          scalar loop (cc_relu)
  LRN           ACROSS_CHANNELS scalar loops (cc_lrn); WITHIN_CHANNEL the
                reference's square / AVE-pool / power / product sub-net
  Pooling       MAX / AVE with padding: scalar loops (cc_pool,
                pooling_layer.cpp:131-200)
  Concat        channel concatenation; Dropout / Split: identity in TEST
  Softmax(WithLoss), Accuracy: softmax (cc_softmax); the loss / accuracy
                scalars are not part of the timed work
Weights are random of the net's shapes (a timing baseline); the Monte-Carlo
map's fault injection runs on the faultable blobs through the C oracle
(oracle.inject, the MC kernel's restatement).
"""
from __future__ import annotations

import re
import time

import numpy as np

import oracle


def parse_prototxt(txt):
    """Minimal text-format parser: {key: [values or nested dicts]}."""
    toks = re.findall(r'"[^"]*"|[{}:]|[^\s{}:"]+', txt)
    pos = 0

    def block():
        nonlocal pos
        d = {}
        while pos < len(toks) and toks[pos] != "}":
            key = toks[pos]
            pos += 1
            if toks[pos] == ":":
                pos += 1
                v = toks[pos]
                pos += 1
                if v.startswith('"'):
                    v = v[1:-1]
                else:
                    try:
                        v = int(v)
                    except ValueError:
                        try:
                            v = float(v)
                        except ValueError:
                            pass
                d.setdefault(key, []).append(v)
            else:  # nested block
                pos += 1  # "{"
                sub = block()
                pos += 1  # "}"
                d.setdefault(key, []).append(sub)
        return d

    return block()


def _one(d, key, default=None):
    v = d.get(key)
    return v[0] if v else default


def _in_phase(layer, phase):
    inc, exc = layer.get("include", []), layer.get("exclude", [])
    if inc and not any(_one(r, "phase") == phase for r in inc):
        return False
    return not any(_one(r, "phase") == phase for r in exc)


class CpuNet:
    """TEST-phase Caffe CPU forward of a prototxt with random weights."""

    def __init__(self, txt, data_shape, batch, seed=0, phase="TEST"):
        net = parse_prototxt(txt)
        self.layers = [l for l in net["layer"] if _in_phase(l, phase)]
        rng = np.random.default_rng(seed)
        shapes = {}
        self.params = {}
        for l in self.layers:
            t = _one(l, "type")
            bots = l.get("bottom", [])
            if t in ("Data", "Input"):
                crop = _one(_one(l, "transform_param", {}), "crop_size")
                ds = tuple(data_shape) if not crop else (data_shape[0], crop, crop)
                self.data_shape = ds
                shapes[l["top"][0]] = (batch,) + ds
                if len(l["top"]) > 1:
                    shapes[l["top"][1]] = (batch,)
                continue
            x = shapes[bots[0]] if bots else None
            if t == "Convolution":
                cp = _one(l, "convolution_param")
                co, k = _one(cp, "num_output"), _one(cp, "kernel_size")
                s, p, g = _one(cp, "stride", 1), _one(cp, "pad", 0), _one(cp, "group", 1)
                w = (rng.standard_normal((co, x[1] // g, k, k)) * 0.01).astype(np.float32)
                b = np.zeros(co, np.float32) if _one(cp, "bias_term", "true") != "false" else None
                self.params[_one(l, "name")] = [w] + ([b] if b is not None else [])
                y = (x[0], co, oracle.out_size(x[2], k, p, s), oracle.out_size(x[3], k, p, s))
            elif t == "InnerProduct":
                co = _one(_one(l, "inner_product_param"), "num_output")
                kin = int(np.prod(x[1:]))
                self.params[_one(l, "name")] = [(rng.standard_normal((co, kin)) * 0.01).astype(np.float32),
                                                np.zeros(co, np.float32)]
                y = (x[0], co)
            elif t == "Pooling":
                pp = _one(l, "pooling_param")
                k, s, p = _one(pp, "kernel_size"), _one(pp, "stride", 1), _one(pp, "pad", 0)
                y = (x[0], x[1], oracle.pool_out(x[2], k, p, s), oracle.pool_out(x[3], k, p, s))
            elif t == "Concat":
                y = (x[0], sum(shapes[b][1] for b in bots)) + tuple(x[2:])
            elif t in ("SoftmaxWithLoss", "Accuracy"):
                y = ()
            else:
                y = x
            for top in l.get("top", []):
                shapes[top] = y
        self.shapes = shapes

    def faultable(self, types=("InnerProduct",)):
        """(layer name, blob index) of the faultable blobs in net order."""
        out = []
        for l in self.layers:
            if _one(l, "type") in types:
                out += [(_one(l, "name"), j) for j in range(len(self.params[_one(l, "name")]))]
        return out

    def forward(self, x, times=None):
        blobs = {}
        out = None
        for l in self.layers:
            t, name = _one(l, "type"), _one(l, "name")
            bots, tops = l.get("bottom", []), l.get("top", [])
            if t in ("Data", "Input"):
                blobs[tops[0]] = x
                continue
            s = time.perf_counter()
            if t == "Convolution":
                cp = _one(l, "convolution_param")
                w = self.params[name]
                y = oracle.cc_conv(blobs[bots[0]], w[0], w[1] if len(w) > 1 else None, _one(cp, "stride", 1),
                                   _one(cp, "pad", 0), _one(cp, "group", 1))
            elif t == "InnerProduct":
                w = self.params[name]
                y = oracle.cc_ip(blobs[bots[0]].reshape(len(x), -1), w[0], w[1])
            elif t == "ReLU":
                y = oracle.cc_relu(blobs[bots[0]])
            elif t == "LRN":
                lp = _one(l, "lrn_param")
                size, a, b = _one(lp, "local_size", 5), _one(lp, "alpha", 1.0), _one(lp, "beta", 0.75)
                if _one(lp, "norm_region") == "WITHIN_CHANNEL":
                    # lrn_layer.cpp WithinChannelForward: square -> AVE pool
                    # (size, pad (size-1)/2, stride 1) -> power -> product
                    xi = blobs[bots[0]]
                    avg = oracle.cc_pool(xi * xi, size, 1, (size - 1) // 2, "AVE")
                    y = (xi * np.power(np.float32(1.0) + np.float32(a) * avg, np.float32(-b))).astype(np.float32)
                else:
                    y = oracle.cc_lrn(blobs[bots[0]], size, a, b, _one(lp, "k", 1.0))
            elif t == "Pooling":
                pp = _one(l, "pooling_param")
                k, st, p = _one(pp, "kernel_size"), _one(pp, "stride", 1), _one(pp, "pad", 0)
                method = _one(pp, "pool", "MAX")
                y = oracle.cc_pool(blobs[bots[0]], k, st, p, method)
            elif t == "Concat":
                y = np.concatenate([blobs[b] for b in bots], axis=1)
            elif t in ("Softmax", "SoftmaxWithLoss"):
                y = oracle.cc_softmax(blobs[bots[0]])
                out = y
            elif t == "Accuracy":
                continue
            else:  # Dropout, Split: identity in TEST
                y = blobs[bots[0]]
            if times is not None:
                times[t] = times.get(t, 0.0) + time.perf_counter() - s
            for top in tops:
                blobs[top] = y
        return out


def mc_map_sample(txt, data_shape, batch, cfgs, seed=0, budget_s=10.0, threads=None, max_images=None):
    """One Monte-Carlo map in Caffe CPU mode on a bounded sample: the map's
    injection into every faultable blob (oracle.inject, cfgs[i] per blob in
    net order), then single-image forwards until `budget_s` is spent (at least
    two); images/s extrapolated to one `batch`-image map.  Returns (images/s,
    metadata)."""
    blas = oracle.cc_init(threads or oracle.physical_cores())
    net = CpuNet(txt, data_shape, 1, seed=seed)
    fl = net.faultable()
    t0 = time.perf_counter()
    broken = 0
    for i, (name, j) in enumerate(fl):
        w = net.params[name][j]
        net.params[name][j], nb = oracle.inject(w.reshape(-1), cfgs[min(i, len(cfgs) - 1)], seed, 0, i)
        net.params[name][j] = net.params[name][j].reshape(w.shape)
        broken += nb
    t_inject = time.perf_counter() - t0
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((1,) + net.data_shape) * 50).astype(np.float32)
    net.forward(x)  # warm the BLAS pool, untimed
    times = {}
    n, t1 = 0, time.perf_counter()
    while n < 2 or (time.perf_counter() - t1 < budget_s and (max_images is None or n < max_images)):
        net.forward(x, times)
        n += 1
    t_img = (time.perf_counter() - t1) / n
    meta = dict(blas=blas, threads=threads or oracle.physical_cores(), images=n, t_inject=t_inject, t_img=t_img,
                broken=broken, faultable_weights=int(sum(net.params[a][b].size for a, b in fl)),
                layer_share={k: round(v / max(sum(times.values()), 1e-12), 3) for k, v in times.items()})
    return batch / (t_inject + batch * t_img), meta
