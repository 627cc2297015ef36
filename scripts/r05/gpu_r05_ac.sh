#!/bin/bash
# r05ac: where the overlapped injection (RRAM_MC_OVERLAP=1) is released:
# after conv1 (this tree, grid 512; lib_g256 grid 256), before conv2
# (lib_b2g256 / lib_b2g512) or after conv2 (lib_a2g256), vs the serial default.
set -o pipefail
O=gpurun_out/r05ac; mkdir -p $O
L=$GRAFT_REPO_ROOT/rram-caffe-simulation_amd
RRAM_LIB_DIR=$L/lib_b2g256 timeout -k 10 300 python -u -m pytest tests/test_gpu_wpack.py -m gpu -x -q --timeout 240 --timeout-method thread -k overlap > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
REPS=3 scripts/ab.sh - "RRAM_MC_OVERLAP=1 RRAM_LIB_DIR=$L/lib_g256" "RRAM_MC_OVERLAP=1 RRAM_LIB_DIR=$L/lib_b2g256" "RRAM_MC_OVERLAP=1 RRAM_LIB_DIR=$L/lib_b2g512" "RRAM_MC_OVERLAP=1 RRAM_LIB_DIR=$L/lib_a2g256" || exit 1
echo done
