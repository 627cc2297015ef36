#!/bin/bash
# conv2 cb16 5x5 per-image tiles at one (OCC=1, no spill) vs two workgroups per CU.
set -o pipefail
O=gpurun_out/r04p2; mkdir -p $O
timeout -k 10 600 env RRAM_CB_OCC1=1 python -u -m pytest tests/test_gpu_fp32_guard.py tests/test_gpu_kernels.py -m gpu -x -q -k "conv2 or engine or conv_patch" --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -40; exit $rc; }
REPS=3 bash scripts/ab.sh - "RRAM_CB_OCC1=1" || exit 1
