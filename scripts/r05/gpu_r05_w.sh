#!/bin/bash
# r05w: pooled-output fold guard tests (a second reader keeps the fp32 top).
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py -k "pooled_output or folded" -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $rc; }
echo done
