#!/bin/bash
# Env-knob A/B on the kbench GEMM shapes: `ENVS="X=0 X=1 X=2" scripts/gpu_envab.sh`
# (each setting run twice, interleaved; base library).
set -o pipefail
O=gpurun_out/envab
mkdir -p $O
for rep in 1 2; do
for e in ${ENVS}; do
  env $e timeout -k 10 120 python scripts/kbench.py --only gemm > $O/kb_${e}_$rep.log 2>&1 || { echo "fail $e"; tail -5 $O/kb_${e}_$rep.log; exit 1; }
  echo "$e.$rep $(grep -E '_ms' $O/kb_${e}_$rep.log | awk '{printf "%s=%s ", $1, $2}')"
done
done
