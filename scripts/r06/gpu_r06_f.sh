#!/bin/bash
# r06f: persistence policy of k_conv_cb16_x6, one-box interleaved A/B:
#   base     = HEAD tree: persistent only when tiles <= 1.5 x the 512 slots (AlexNet conv5)
#   lib_np   = RRAM_CB16_PERSIST_X2=0: the loop kernel, one tile per workgroup everywhere
#   lib_pall = RRAM_CB16_PERSIST_X2=100: persistent everywhere (r06e's build)
#   lib_head = e54205b: the non-persistent kernel
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_octets.py \
  tests/test_gpu_fp32_guard.py > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/rram-caffe-simulation_amd
REPS=2 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_np" "RRAM_LIB_DIR=$L/lib_pall" "RRAM_LIB_DIR=$L/lib_head" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
