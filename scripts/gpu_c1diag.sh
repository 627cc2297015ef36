#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
for d in 0 1 2 4 8 15; do
  RRAM_C1_DIAG=$d timeout -k 10 120 python scripts/conv1_check.py > $O/c1d_$d.json 2>&1
  echo "diag $d: $(tail -1 $O/c1d_$d.json)"
done
