#!/bin/bash
# GEMM split-K sweep: RRAM_GEMM_SPLIT_MINK x RRAM_GEMM_SPLIT_TARGET (default 256 x 256)
set -o pipefail
O=gpurun_out/r04ao; mkdir -p $O
for rep in 1 2; do for cfg in "256 256" "128 256" "256 512"; do set -- $cfg; for w in lenet_mc lenet_train cifar10_quick_mc cifar10_full_train alexnet_mc; do
  RRAM_GEMM_SPLIT_MINK=$1 RRAM_GEMM_SPLIT_TARGET=$2 timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('mink=$1 target=$2 $w', d['value'], d['ms_per_step'])"
done; done; done
