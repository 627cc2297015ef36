#!/bin/bash
# overlapped injection grid A/B (RRAM_INJECT_GRID)
set -o pipefail
O=gpurun_out/injgrid
mkdir -p $O
for r in 1 2; do for g in 2048 512 128; do
  RRAM_INJECT_GRID=$g timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/b_${g}_$r.json 2> $O/l_${g}_$r.txt || exit 1
  echo "grid=$g $(grep -o '"value": [0-9.]*' $O/b_${g}_$r.json) inj_us=$(python3 -c "import json; print(json.load(open('$O/b_${g}_$r.json'))['roofline_inject']['avg_us_per_launch'])") $(grep -E 'conv1 ' $O/l_${g}_$r.txt | tr -s ' ')"
done; done
