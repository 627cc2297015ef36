#!/bin/bash
# octet companions: none (0) / all producers (1) / LRN+pool only (2, default)
set -o pipefail
O=gpurun_out/octmode
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_octets.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "octet or c3 or alexnet" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for m in 0 2 1; do
  RRAM_OCTETS=$m timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/b_${m}_$r.json 2> $O/l_${m}_$r.txt || exit 1
  echo "octets=$m $(grep -o '"value": [0-9.]*' $O/b_${m}_$r.json) $(grep -E 'conv[2-5] |pool[12] ' $O/l_${m}_$r.txt | tr -s ' ' | tr '\n' ' ')"
done; done
