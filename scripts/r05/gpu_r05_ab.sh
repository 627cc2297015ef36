#!/bin/bash
# r05ab: the overlapped injection (RRAM_MC_OVERLAP=1) released after conv1
# (this tree) vs released with the prefix (lib_rel0), and its grid (512 here;
# lib_g256 / lib_g1024), against the serial default: overlap parity test,
# then the interleaved A/B.
set -o pipefail
O=gpurun_out/r05ab; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_wpack.py -m gpu -x -q --timeout 240 --timeout-method thread -k overlap > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
REPS=3 scripts/ab.sh - "RRAM_MC_OVERLAP=1" "RRAM_MC_OVERLAP=1 RRAM_LIB_DIR=$L/lib_rel0" "RRAM_MC_OVERLAP=1 RRAM_LIB_DIR=$L/lib_g256" "RRAM_MC_OVERLAP=1 RRAM_LIB_DIR=$L/lib_g1024" || exit 1
echo done
