#!/bin/bash
# r05aa: conv5 on 128 x 64 tiles at two per CU (lib_n64: 1352 workgroups,
# 2.6 rounds of 512) vs 128 x 128 (this tree: 676 workgroups, the second of
# two rounds a third full): octet + fp32-guard tests, interleaved A/B.
set -o pipefail
O=gpurun_out/r05aa; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
RRAM_LIB_DIR=$L/lib_n64 timeout -k 10 400 python -u -m pytest tests/test_gpu_octets.py tests/test_gpu_fp32_guard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
REPS=3 scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_n64" || exit 1
echo done
