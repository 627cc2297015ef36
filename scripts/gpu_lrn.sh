#!/bin/bash
# LRN + max-pool channels per barrier (RRAM_LRN_G) A/B, with its parity tests
set -o pipefail
O=gpurun_out/lrn
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_octets.py tests/test_gpu_layers.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lrn or pool or c3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in 2 4 8; do for r in 1 2; do
  RRAM_LRN_G=$g RRAM_X6=1 timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers --steps 10 > $O/b_${g}_$r.json 2> $O/l_${g}_$r.txt || exit 1
  echo "G=$g $(grep -o '"value": [0-9.]*' $O/b_${g}_$r.json) $(grep -E 'pool[12] ' $O/l_${g}_$r.txt | tr -s ' ' | tr '\n' ' ')"
done; done
