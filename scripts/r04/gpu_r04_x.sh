#!/bin/bash
# per-shape data-gradient A/B (scripts/dx_ab.py)
set -o pipefail
O=gpurun_out/r04x; mkdir -p $O
for v in 0 1; do
  timeout -k 10 300 env RRAM_DX_FWD=$v python -u scripts/dx_ab.py > $O/dx_$v.jsonl 2> $O/dx_$v.err || { tail -5 $O/dx_$v.err; exit 1; }
done
python3 - <<'PY'
import json
a = {(r["engine"], r["shape"]): r["us"] for r in map(json.loads, open("gpurun_out/r04x/dx_0.jsonl"))}
b = {(r["engine"], r["shape"]): r["us"] for r in map(json.loads, open("gpurun_out/r04x/dx_1.jsonl"))}
for k in a:
    print(f"{k[0]:7s} {k[1]:12s} col2im {a[k]:8.1f} us  flipped-fwd {b[k]:8.1f} us  ratio {b[k]/a[k]:.2f}")
PY
