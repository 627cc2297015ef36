#!/bin/bash
# r06j: k_conv_cb16_x6 skips the MFMAs of column blocks wholly past a per-image tile's last position
# (AlexNet conv2: 89 of the sixth tile's 128 columns are positions); tests first, then an interleaved
# A/B against lib_noskip (RRAM_CB16_SKIPJ=0).
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_octets.py \
  tests/test_gpu_fp32_guard.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_wpack.py \
  tests/test_gpu_layers.py > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/rram-caffe-simulation_amd
REPS=3 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_noskip" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
