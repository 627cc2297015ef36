#!/bin/bash
# MC injection overlapped with conv1-5 on a side stream (RRAM_MC_OVERLAP=1) vs serial
set -o pipefail
O=gpurun_out/mcov
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b0_$r.json 2> $O/e0_$r.txt || exit 1
  RRAM_MC_OVERLAP=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b1_$r.json 2> $O/e1_$r.txt || exit 1
  echo "serial $(grep -o '"value": [0-9.]*' $O/b0_$r.json)  overlap $(grep -o '"value": [0-9.]*' $O/b1_$r.json)"
done
RRAM_MC_OVERLAP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mc or MC or monte" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
