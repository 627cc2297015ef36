#!/bin/bash
# weight-gradient split-K up to 256 (>= 256 K per split) + wave-per-output reduce for >= 32 splits;
# A/B: RRAM_DW_SPLIT_CAP=64 RRAM_DW_SPLIT_MINK=512 (the old split; the reduce is the new one either way)
set -o pipefail
O=gpurun_out/r04am; mkdir -p $O
true || timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_solver_kat.py tests/test_gpu_host.py tests/test_gpu_parallel.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_k.log 2>&1; rc=$?
tail -2 $O/tests_k.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_k.log | head -40; exit $rc; }
for rep in 1 2; do for cfg in "256 256" "512 128" "1024 64"; do set -- $cfg; for w in cifar10_full_train lenet_train; do
  RRAM_DW_SPLIT_CAP=$1 RRAM_DW_SPLIT_MINK=$2 timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('cap=$1 mink=$2 $w', d['value'], d['ms_per_step'])"
done; done; done
