#!/bin/bash
# conv1 compact-K check: conv1 tests, then bench layer table + conv1 PMC.
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wpack.py tests/test_gpu_fp32_guard.py tests/test_gpu_layers.py tests/test_gpu_configs.py -k "conv1 or engine or c3 or c5 or alexnet or strided or cached or mc_maps or fp32_level or pool" -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "err / sum|conv1" $O/tests.log | head -5; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
REPS=2 bash scripts/ab.sh - || exit 1
mkdir -p gpurun_out/pmcab && KF="conv1|cb" bash scripts/gpu_pmc_ab.sh - || exit 1
grep -E "conv1_ring" gpurun_out/pmcab/v1.txt | cut -c1-700
timeout -k 10 300 python -u scripts/gn_layers.py > $O/gn_layers.txt 2>&1 && head -60 $O/gn_layers.txt
