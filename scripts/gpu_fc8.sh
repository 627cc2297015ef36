#!/bin/bash
# fc8 on the x6 GEMM (RRAM_X6_GEMM_MINWG=128) vs the fp32 kernel (192)
set -o pipefail
O=gpurun_out/fc8
mkdir -p $O
for r in 1 2; do for m in 192 128; do
  RRAM_X6_GEMM_MINWG=$m timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers --steps 10 > $O/b_${m}_$r.json 2> $O/l_${m}_$r.txt || exit 1
  echo "minwg=$m $(grep -o '"value": [0-9.]*' $O/b_${m}_$r.json) $(grep -E 'fc[678] ' $O/l_${m}_$r.txt | tr -s ' ' | tr '\n' ' ')"
done; done
RRAM_X6_GEMM_MINWG=128 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ip or gemm or c3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
