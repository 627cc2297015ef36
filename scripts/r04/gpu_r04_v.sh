#!/bin/bash
# persistent LDS-DMA 1x1 kernel (RRAM_C1X1=4): tests, layer table, C5 A/B vs the default.
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 600 env RRAM_C1X1=4 python -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_octets.py tests/test_gpu_wpack.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -40; exit $rc; }
for v in 4 1; do
  timeout -k 10 300 env RRAM_C1X1=$v python -u scripts/gn_layers.py --top 70 > $O/gn_$v.txt 2>&1 || { tail -5 $O/gn_$v.txt; exit 1; }
  head -2 $O/gn_$v.txt | tail -1
done
for v in 4 1 4 1; do
  timeout -k 10 300 env RRAM_C1X1=$v python bench.py --workload googlenet_sweep --steps 5 --warmup 1 --no-cpu-baseline > $O/c5_$v.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json')); print('C5 c1x1=$v', d['value'], d['ms_per_step'])"
done
