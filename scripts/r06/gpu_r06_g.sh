#!/bin/bash
# r06g: conv1 A/B: lib_c1l = RRAM_C1_LOAD128, the refill's eight 4-byte input
# loads per 8-column chunk as two 16-byte loads (4-byte aligned); its conv1 tests first (C3 conv1
# vs float64, the fp32 guard, the non-finite / range tests), then an interleaved A/B vs the tree.
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
RRAM_LIB_DIR=$PWD/rram-caffe-simulation_amd/lib_c1l timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread "tests/test_gpu_configs.py::test_c3_alexnet_b256_per_layer_fp64" tests/test_gpu_fp32_guard.py \
  tests/test_gpu_x6_range.py tests/test_gpu_layers.py > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/rram-caffe-simulation_amd
REPS=3 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_c1l" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
