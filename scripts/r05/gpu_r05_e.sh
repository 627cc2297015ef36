#!/bin/bash
# r05e: conv1 per-group stamp shares (diagnostic build lib_c1stamp)
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
RRAM_LIB_DIR=$GRAFT_REPO_ROOT/rram-caffe-simulation_amd/lib_c1stamp timeout -k 10 300 python scripts/c1_stamp.py > $O/c1_stamp.txt 2>&1; rc=$?
cat $O/c1_stamp.txt; exit $rc
