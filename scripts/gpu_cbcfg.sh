#!/bin/bash
# A/B of the channel-octet kernel's tile (RRAM_CB_CFG) on the bench's per-layer times.
set -o pipefail
O=gpurun_out/cbcfg
mkdir -p $O
for r in 1 2; do
for cfg in "" "4,8" "4,4" "2,4"; do
  RRAM_CB_CFG=$cfg timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/b_${cfg}_$r.json 2> $O/l_${cfg}_$r.txt || exit 1
  echo "[$cfg] $(grep -o '"value": [0-9.]*' $O/b_${cfg}_$r.json)"; grep -E "conv[2-5] " $O/l_${cfg}_$r.txt | tr -s ' ' | tr '\n' ' '; echo
done
done
