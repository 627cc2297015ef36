#!/bin/bash
# r06i: conv1 A/B: lib_c1s = RRAM_C1_SPREAD, the slot refill one 8-column chunk per group over five
# consecutive groups per slot (load, store one group later) instead of two chunks on every other group
# (483 VGPRs, no scratch, vs 512 + 20 B); its conv1 tests first, then an interleaved A/B vs the tree.
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
RRAM_LIB_DIR=$PWD/rram-caffe-simulation_amd/lib_c1s timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread "tests/test_gpu_configs.py::test_c3_alexnet_b256_per_layer_fp64" tests/test_gpu_fp32_guard.py \
  tests/test_gpu_x6_range.py tests/test_gpu_layers.py > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/rram-caffe-simulation_amd
REPS=3 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_c1s" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
