#!/bin/bash
# TRAIN softmax loss fwd+bwd in one launch; tiny GEMMs without split-K (A/B RRAM_GEMM_SPLIT_MIN_MFLOP);
# MonteCarlo statistics folded into the Accuracy / SoftmaxWithLoss stores
set -o pipefail
O=gpurun_out/r04ak; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_all.log 2>&1; rc=$?
tail -2 $O/tests_all.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_all.log | head -40; exit $rc; }
for rep in 1 2; do for mf in 32 0; do for w in cifar10_quick_mc cifar10_full_train lenet_mc lenet_train; do
  RRAM_GEMM_SPLIT_MIN_MFLOP=$mf timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('minmflop=$mf $w', d['value'], d['ms_per_step'])"
done; done; done
