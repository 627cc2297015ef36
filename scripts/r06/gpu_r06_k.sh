#!/bin/bash
# r06k: where the 3x3 octet kernel's cycles go -- diagnostic builds of k_conv_cb16_x6 each leaving out
# parts of its loop (RRAM_CB16_ABLATE bit mask: 1 B reads, 2 weight loads, 4 patch staging, 8 barriers,
# 16 epilogue stores, 31 all of them; results wrong, timing only), interleaved with the product build.
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
L=$PWD/rram-caffe-simulation_amd
REPS=2 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_a1" "RRAM_LIB_DIR=$L/lib_a2" "RRAM_LIB_DIR=$L/lib_a4" \
  "RRAM_LIB_DIR=$L/lib_a8" "RRAM_LIB_DIR=$L/lib_a16" "RRAM_LIB_DIR=$L/lib_a31" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
