#!/bin/bash
# overlapped injection start (RRAM_MC_INJECT_AFTER: layers run before it starts)
set -o pipefail
O=gpurun_out/injafter
mkdir -p $O
for r in 1 2; do for k in 0 3 6; do
  RRAM_MC_INJECT_AFTER=$k timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/b_${k}_$r.json 2> $O/l_${k}_$r.txt || exit 1
  echo "after=$k $(grep -o '"value": [0-9.]*' $O/b_${k}_$r.json) inj_us=$(python3 -c "import json; print(json.load(open('$O/b_${k}_$r.json'))['roofline_inject']['avg_us_per_launch'])") $(grep -E 'conv[12] ' $O/l_${k}_$r.txt | tr -s ' ' | tr '\n' ' ')"
done; done
RRAM_MC_INJECT_AFTER=6 timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mc or MC" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
