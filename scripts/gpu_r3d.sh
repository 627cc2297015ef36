#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wpack.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_r3d.log 2>&1; rc=$?
tail -3 $O/pytest_r3d.log; [ $rc -eq 0 ] || exit $rc
REPS=1 ./scripts/ab.sh - RRAM_LRN_BLOCKS=2048 RRAM_LRN_BLOCKS=8192 RRAM_LRN_BLOCKS=16384 || exit 1
