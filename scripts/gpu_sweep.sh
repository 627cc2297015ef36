#!/bin/bash
# GEMM tuning sweep over the RRAM_GEMM_KB / RRAM_GEMM_TILE knobs (kbench conv + IP times).
set -o pipefail
O=gpurun_out/sweep
mkdir -p $O
for kb in 32 16; do
  for t in 0 128 192 96 64 6464; do
    RRAM_GEMM_KB=$kb RRAM_GEMM_TILE=$t timeout -k 10 120 python scripts/kbench.py --only gemm > $O/kb_${kb}_${t}.log 2>&1 || { echo "fail kb=$kb t=$t"; tail -5 $O/kb_${kb}_${t}.log; exit 1; }
    echo "kb=$kb tile=$t $(grep -E '_ms' $O/kb_${kb}_${t}.log | awk '{printf "%s=%s ", $1, $2}')"
  done
done
