#!/bin/bash
# TRAIN-phase softmax loss forward + backward in one launch; no split-K for tiny GEMMs (A/B RRAM_GEMM_SPLIT_MIN_MFLOP)
set -o pipefail
O=gpurun_out/r04aj; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_layers.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_solver_kat.py tests/test_gpu_host.py tests/test_gpu_ref_kats.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_k.log 2>&1; rc=$?
tail -2 $O/tests_k.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_k.log | head -40; exit $rc; }
for rep in 1 2; do for mf in 32 0; do for w in cifar10_quick_mc cifar10_full_train lenet_train; do
  RRAM_GEMM_SPLIT_MIN_MFLOP=$mf timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('minmflop=$mf $w', d['value'], d['ms_per_step'])"
done; done; done
