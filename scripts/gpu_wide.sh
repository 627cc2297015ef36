#!/bin/bash
# conv1 (k_conv_wide_x6) weights from L2 (RRAM_WIDE_GA=1) vs the LDS ring (0):
# conv parity tests, then the bench's per-layer times, two rounds.
set -o pipefail
O=gpurun_out/wide
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -m gpu -x -q -rP --timeout 300 --timeout-method thread -k "engine or conv or c3" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log; grep "227, 227" $O/pytest.log | head -2
for r in 1 2; do for x in 0 1; do
  RRAM_WIDE_GA=$x timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/b_${x}_$r.json 2> $O/l_${x}_$r.txt || exit 1
  echo "GA=$x $(grep -o '"value": [0-9.]*' $O/b_${x}_$r.json) $(grep -E 'conv1 ' $O/l_${x}_$r.txt | tr -s ' ')"
done; done
