#!/bin/bash
# r05v: hipGraph-replayed AlexNet maps with the pooled-output fold, pool1 read
# between runs (the fold undone -> recapture), vs eager; plus the graph and
# layer test files.
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_layers.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $rc; }
echo done
