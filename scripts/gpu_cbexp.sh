#!/bin/bash
# diagnostic timing of k_conv_cb_x6 with parts of its loop removed (RRAM_CB_EXP bits)
set -o pipefail
O=gpurun_out/cbexp
mkdir -p $O
for e in 0 1 2 3 4 7 0; do
  RRAM_CB_EXP=$e timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers --steps 10 > $O/b_$e.json 2> $O/l_$e.txt || exit 1
  echo "exp=$e $(grep -E 'conv[2-5] ' $O/l_$e.txt | tr -s ' ' | tr '\n' ' ')"
done
