#!/bin/bash
# A/B: octet companions written by the producers (RRAM_OCTETS=1) vs packed
# by each convolution (0) vs the patch kernels (RRAM_CONV_CB=0); 2 rounds.
set -o pipefail
O=gpurun_out/octab
mkdir -p $O
for r in 1 2; do
for cfg in "RRAM_OCTETS=1" "RRAM_OCTETS=0" "RRAM_CONV_CB=0"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/b_${cfg}_$r.json 2> $O/l_${cfg}_$r.txt || exit 1
  echo "$cfg $(cut -c1-150 $O/b_${cfg}_$r.json | grep -o '"value": [0-9.]*')"; grep -E "conv[2-5] |pool[12] " $O/l_${cfg}_$r.txt | tr -s ' ' | tr '\n' ' '; echo
done
done
