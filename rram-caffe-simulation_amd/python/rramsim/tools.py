"""Experiment tools of the fork, re-expressed for this build.

prune_order — examples/cifar10/gaussian_failure/prune_order.py:30-49: magnitude
prune every FC layer ("fc*" layers, weights only) at `prune_ratio`, then for
each adjacent FC pair rank the neurons of layer i-1 by (#zero weights in their
input row + #zero weights in their output column) — the order the remapping
strategy reads from its prune_order_file (strategy.hpp:104-123).  Host numpy,
like the reference script; np.argsort's default kind matches it tie for tie.

Usage:  python -m rramsim.tools prune_order NET.prototxt WEIGHTS.caffemodel RATIO OUT.txt
"""
from __future__ import annotations

import argparse
from typing import List, Sequence, Tuple

import numpy as np


def magnitude_prune(w: np.ndarray, prune_ratio: float) -> np.ndarray:
    """prune_order.py:34-38: zero the int(size * ratio) smallest |w|."""
    flat = np.array(w, dtype=np.float32).reshape(-1)
    rank = np.argsort(np.abs(flat))
    flat[rank[:int(rank.size * prune_ratio)]] = 0
    return flat.reshape(np.shape(w))


def prune_orders(fc_weights: Sequence[np.ndarray], prune_ratio: float) -> Tuple[List[np.ndarray], List[np.ndarray]]:
    """(pruned weights, orders): orders[i-1] ranks the neurons of FC layer i-1
    (prune_order.py:44-49)."""
    pruned = [magnitude_prune(w, prune_ratio) for w in fc_weights]
    orders = []
    for i in range(1, len(pruned)):
        zero_nums = (pruned[i - 1] == 0).astype(np.int64).sum(axis=1) + (pruned[i] == 0).astype(np.int64).sum(axis=0)
        orders.append(np.argsort(zero_nums))
    return pruned, orders


def write_prune_order_file(path: str, orders: Sequence[np.ndarray]) -> None:
    with open(path, "w") as wf:
        for o in orders:
            wf.write(" ".join(str(int(x)) for x in o))
            wf.write("\n")


def experiment_solver(template: str, mean: float, std: float, threshold: float = 0.0, remapping: str = "",
                      genetic: str = "", prob: int = -1, snapshot_prefix: str = "") -> str:
    """SolverParameter text for one fault experiment, as
    examples/cifar10/gaussian_failure/run_gaussian_exp.py:50-103 derives it from
    a template: failure_pattern mean/std; `threshold` > 0 appends a threshold
    strategy; `remapping` = "order_file[,period[,start]]"; `genetic` =
    "prune_net,prune_model[,switch_time[,period[,start]]]"; `prob` >= 0 sets the
    stuck-at split to (prob, 100 - 2 prob, prob)."""
    lines = [l for l in template.splitlines()
             if not l.strip().startswith(("failure_pattern", "snapshot_prefix"))]
    text = "\n".join(lines)
    fp = f"failure_pattern {{ mean: {mean} std: {std}"
    if prob >= 0:
        assert prob < 50
        fp += f" failure_prob {{ neg: {prob} zero: {100 - 2 * prob} pos: {prob} }}"
    out = [text, fp + " }"]
    if snapshot_prefix:
        out.append(f'snapshot_prefix: "{snapshot_prefix}/"')
    if threshold > 0:
        out.append(f'failure_strategy {{ type: "threshold" threshold: {threshold} }}')
    if remapping:
        st = remapping.split(",")
        s_ = f'failure_strategy {{ type: "remapping" prune_order_file: "{st[0]}"'
        if len(st) > 1:
            s_ += f" period: {int(st[1])}"
        if len(st) > 2:
            s_ += f" start: {int(st[2])}"
        out.append(s_ + " }")
    if genetic:
        st = genetic.split(",")
        s_ = f'failure_strategy {{ type: "genetic" prune_net_file: "{st[0]}" prune_model_file: "{st[1]}"'
        for k, key in ((2, "switch_time"), (3, "period"), (4, "start")):
            if len(st) > k:
                s_ += f" {key}: {int(st[k])}"
        out.append(s_ + " }")
    return "\n".join(out) + "\n"


def _fc_weights_of(prototxt_path: str, caffemodel: str, options=None) -> List[np.ndarray]:
    """FC weight matrices ("fc*" layers with params, net order) of a TEST net."""
    from . import caffe
    net = caffe.Net(open(prototxt_path).read(), "test", options)
    net.copy_from(caffemodel)
    ps = net.params()
    out, k = [], 0
    for name, typ, npar in net.layers():
        if npar and name[:2] == "fc":
            w = ps[k]["data"].detach().cpu().numpy()
            out.append(w.reshape(w.shape[0], -1) if w.ndim != 2 else w)
        k += npar
    net.close()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(prog="rramsim.tools")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("prune_order", help="write the remapping strategy's prune order file")
    p.add_argument("proto")
    p.add_argument("model")
    p.add_argument("prune_ratio", type=float)
    p.add_argument("output_file")
    p.add_argument("--data-shape", default=None, help='C,H,W of synthetic Data layers, e.g. "3,32,32"')
    a = ap.parse_args(argv)
    if a.cmd == "prune_order":
        opts = {"data_shape": a.data_shape} if a.data_shape else None
        _, orders = prune_orders(_fc_weights_of(a.proto, a.model, opts), a.prune_ratio)
        write_prune_order_file(a.output_file, orders)
        print(f"proto: {a.proto}; model: {a.model}; prune_ratio: {a.prune_ratio}; output_file: {a.output_file}")


if __name__ == "__main__":
    main()
