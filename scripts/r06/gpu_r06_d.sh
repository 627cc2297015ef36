#!/bin/bash
# r06d: the graph / fold / native-DP GPU tests after the graph-key and
# convolution-output-fold changes, then one-box interleaved A/Bs of the
# headline (scripts/ab.sh, per-layer live events):
#   base   = HEAD (conv3 -> conv4 -> conv5 convolution-output fold on)
#   nocy   = lib_nocy: the fold off (RRAM_CONV_Y_FOLD=0)
#   sd5    = lib_sd5: conv2's 5x5 form at staging distance 1 (RRAM_CB16_SD5=1)
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_layers.py::test_conv_octets_only_epilogue_bit_identical" \
  "tests/test_gpu_layers.py::test_conv_output_fold_materialises" tests/test_gpu_graph.py \
  tests/test_gpu_native_dp.py tests/test_gpu_octets.py \
  "tests/test_gpu_layers.py::test_pooled_output_fold_materialises" > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/rram-caffe-simulation_amd
REPS=3 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_nocy" "RRAM_LIB_DIR=$L/lib_sd5" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
