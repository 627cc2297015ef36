#!/bin/bash
# Env-knob A/B on the headline bench itself (real AlexNet activations, not
# kbench's random operands: the held clock depends on the data):
# `ENVS="X=0 X=1" scripts/gpu_benchab.sh`, each setting twice, interleaved.
# Prints img/s, GEMM TFLOP/s and the conv / fc layer times (hipEvents).
set -o pipefail
O=gpurun_out/benchab
mkdir -p $O
for rep in 1 2; do
for e in ${ENVS}; do
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --profile-layers > $O/b_${e}_$rep.json 2> $O/b_${e}_$rep.err || { echo "fail $e"; tail -5 $O/b_${e}_$rep.err; exit 1; }
  python3 - "$O/b_${e}_$rep.json" "$O/b_${e}_$rep.err" "$e.$rep" <<'PY'
import json, sys, re
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lay = {}
for l in open(sys.argv[2]):
    m = re.match(r"\s*(conv\d|fc\d|pool\d)\s+\S+\s+([\d.]+) ms", l)
    if m: lay[m.group(1)] = float(m.group(2))
print(sys.argv[3], round(b["value"]), b["roofline"]["achieved"], " ".join(f"{k}={v:.3f}" for k, v in lay.items()))
PY
done
done
