#!/bin/bash
# k_conv_cb_x6 loads: compiler-visible register loads (RRAM_CB_VL=1) vs LDS-DMA ring (0)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/vl
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_octets.py tests/test_gpu_kernels.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "octet or patch or engine or conv or c3" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for x in 0 1; do
  RRAM_CB_VL=$x timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/b_${x}_$r.json 2> $O/l_${x}_$r.txt || exit 1
  echo "VL=$x $(grep -o '"value": [0-9.]*' $O/b_${x}_$r.json) $(grep -E 'conv[2-5] ' $O/l_${x}_$r.txt | tr -s ' ' | tr '\n' ' ')"
done; done
