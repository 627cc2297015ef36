#!/bin/bash
# r05f: octet-kernel plans at two workgroups per CU (conv3 128x128, conv4 /
# conv5 64x128: lib) vs r05d's lib_occ2 (conv3 only); conv1 stamp shares.
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
T="tests/test_gpu_octets.py tests/test_gpu_fp32_guard.py tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_wpack.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_occ2" - || exit 1
RRAM_LIB_DIR=$L/lib_c1stamp timeout -k 10 300 python scripts/c1_stamp.py > $O/c1_stamp.txt 2>&1 || exit 1
cat $O/c1_stamp.txt
echo done
