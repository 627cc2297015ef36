#!/bin/bash
# ReLU folded into the Pooling store (rram_pool_relu_fwd); C2 / C4 / C1 re-measured.
set -o pipefail
O=gpurun_out/r04ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_configs.py tests/test_gpu_graph.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_k.log 2>&1; rc=$?
tail -2 $O/tests_k.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_k.log | head -40; exit $rc; }
for w in cifar10_quick_mc cifar10_full_train lenet_mc lenet_train cifar10_quick_mc cifar10_full_train; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', d['value'], d['ms_per_step'])"
done
