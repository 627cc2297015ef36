#!/bin/bash
# split-K for IP / GEMMs from K >= 256 (>= 128 K per split); A/B RRAM_GEMM_SPLIT_MINK=1024 (rounds 1-4)
set -o pipefail
O=gpurun_out/r04an; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_host.py tests/test_gpu_solver_kat.py tests/test_gpu_ref_kats.py tests/test_gpu_layers.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_k.log 2>&1; rc=$?
tail -2 $O/tests_k.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_k.log | head -40; exit $rc; }
for rep in 1 2; do for mk in 256 1024; do for w in lenet_mc lenet_train cifar10_quick_mc cifar10_full_train; do
  RRAM_GEMM_SPLIT_MINK=$mk timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('mink=$mk $w', d['value'], d['ms_per_step'])"
done; done; done
