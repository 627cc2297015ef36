#!/bin/bash
# C4: the solver tail in one launch (rram_fused_update_fail_batched); conv bias gradient in one launch.
set -o pipefail
O=gpurun_out/r04z2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_host.py -m gpu -x -q -k "fused or tail or c4 or solver or graph or bias or bwd" --timeout 120 --timeout-method thread > $O/tests_k.log 2>&1; rc=$?
tail -2 $O/tests_k.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_k.log | head -40; exit $rc; }
for w in cifar10_full_train lenet_train cifar10_full_train lenet_train; do
  timeout -k 10 300 python bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('$w', d['value'], d['ms_per_step'])"
done
