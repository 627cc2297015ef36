#!/bin/bash
# 1x1 x6 kernel: tests, then GoogLeNet layer table and C5 with / without it.
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_wpack.py tests/test_gpu_configs.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -40; exit $rc; }
for v in 1 0; do
  timeout -k 10 300 env RRAM_C1X1=$v python -u scripts/gn_layers.py --top 70 > $O/gn_layers_c1x1_$v.txt 2>&1 || { tail -5 $O/gn_layers_c1x1_$v.txt; exit 1; }
  head -2 $O/gn_layers_c1x1_$v.txt | tail -1
done
for v in 1 0 1 0; do
  timeout -k 10 300 env RRAM_C1X1=$v python bench.py --workload googlenet_sweep --steps 5 --warmup 1 --no-cpu-baseline > $O/c5_$v.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json')); print('C5 c1x1=$v', d['value'], d['ms_per_step'], d['roofline'].get('achieved'))"
done
for w in cifar10_quick_mc lenet_mc cifar10_full_train; do
  for sg in "0 0" "0 1" "1 0" "1 1"; do
    set -- $sg
    timeout -k 10 300 env RRAM_BENCH_STREAM=$1 RRAM_MC_GRAPH=$2 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/${w}_s$1g$2.json 2> $O/${w}_s$1g$2.err || { tail -5 $O/${w}_s$1g$2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${w}_s$1g$2.json')); print('$w stream=$1 graph=$2', d['value'], d['unit'], d['ms_per_step'], d.get('hipgraph'))"
  done
done
