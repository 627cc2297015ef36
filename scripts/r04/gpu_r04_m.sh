#!/bin/bash
# 1x1 octet-companion epilogue: tests, GoogLeNet layer table + C5.
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_octets.py tests/test_gpu_conv1x1.py tests/test_gpu_configs.py tests/test_gpu_layers.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -40; exit $rc; }
timeout -k 10 300 python -u scripts/gn_layers.py --top 70 > $O/gn_layers.txt 2>&1 || { tail -5 $O/gn_layers.txt; exit 1; }
head -2 $O/gn_layers.txt | tail -1
for v in 1 1; do
  timeout -k 10 300 python bench.py --workload googlenet_sweep --steps 5 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5.json')); print('C5', d['value'], d['ms_per_step'], d['roofline'].get('achieved'))"
done
