"""Per-layer hipEvent times of the C5 workload (GoogLeNet b256 TEST forward
under a fault map), with each contraction's TFLOP/s against the bf16x6 roof.
Diagnostic only: prints one table, sorted by time, and the per-type totals.

  python scripts/gn_layers.py [--maps 6] [--batch 256]
"""
import argparse
import os
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "rram-caffe-simulation_amd" / "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--maps", type=int, default=6)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import torch
    from rramsim import caffe, make_inject_cfg, models
    torch.cuda.init()
    fold = os.environ.get("RRAM_FUSE_CONCAT", "1") != "0"
    net = caffe.Net(models.googlenet(test_batch=a.batch), "test", models.net_options("googlenet", fuse_concat=fold))
    mc = caffe.MonteCarlo(net, make_inject_cfg(0.01), seed=5, max_maps=a.maps + 4)
    for i in range(2):
        mc.run(i, 1)
    torch.cuda.synchronize()
    net.layer_times(reset=True)
    net.set_timing(1)
    for i in range(a.maps):
        mc.run(2 + i, 1)
    torch.cuda.synchronize()
    net.set_timing(0)
    lt = net.layer_times(reset=True)
    con = net.contractions()
    tot = sum(m for _, _, m, _ in lt) / a.maps
    by_type = defaultdict(float)
    rows = []
    for name, typ, ms, cnt in lt:
        if cnt == 0:
            continue
        per = ms / a.maps
        by_type[typ] += per
        tf = ""
        if name in con:
            tf = f"{con[name][0] / (per * 1e-3) / 1e12:7.1f}"
        rows.append((per, name, typ, tf))
    rows.sort(reverse=True)
    print(f"GoogLeNet b{a.batch} TEST, fold={int(fold)}: {tot:.3f} ms per map (sum of layer events)")
    for per, name, typ, tf in rows[:a.top]:
        print(f"  {name:40s} {typ:14s} {per * 1e3:9.1f} us {tf:>8s} TFLOP/s")
    print("per type:")
    for typ, v in sorted(by_type.items(), key=lambda kv: -kv[1]):
        print(f"  {typ:14s} {v:8.3f} ms  {100 * v / tot:5.1f} %")
    mc.close()
    net.close()


if __name__ == "__main__":
    main()
