#!/bin/bash
# gather kernel (GoogLeNet conv1 on bf16x6): tests, layer table, C5 A/B.
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_wpack.py tests/test_gpu_configs.py tests/test_abi.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "gather|conv1/7x7" $O/tests.log | head; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -40; exit $rc; }
for v in 1 0; do
  timeout -k 10 300 env RRAM_GATHER_X6=$v python -u scripts/gn_layers.py --top 12 > $O/gn_$v.txt 2>&1 || { tail -5 $O/gn_$v.txt; exit 1; }
  head -2 $O/gn_$v.txt | tail -1; grep "conv1/7x7" $O/gn_$v.txt
done
for v in 1 0 1 0; do
  timeout -k 10 300 env RRAM_GATHER_X6=$v python bench.py --workload googlenet_sweep --steps 5 --warmup 1 --no-cpu-baseline > $O/c5_$v.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json')); print('C5 gather=$v', d['value'], d['ms_per_step'], d['roofline'].get('achieved'))"
done
