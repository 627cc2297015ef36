#!/bin/bash
# r06e: the persistent k_conv_cb16_x6 (next tile's patch / first weights
# prefetched under the epilogue): octet / fp32-guard / config tests, then a
# one-box interleaved A/B against lib_head (= e54205b, non-persistent).
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_octets.py \
  tests/test_gpu_fp32_guard.py "tests/test_gpu_layers.py::test_conv_output_fold_materialises" \
  "tests/test_gpu_layers.py::test_conv_octets_only_epilogue_bit_identical" tests/test_gpu_configs.py \
  tests/test_gpu_graph.py > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/rram-caffe-simulation_amd
REPS=3 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_head" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
