#!/bin/bash
# r05d: 2-tap patch staging in k_conv_cb_x6 (lib) and conv3 on the 16x16x32
# form at two workgroups per CU (lib_occ2, -DRRAM_CB_PREFER_OCC2): octet /
# guard / kernel tests on both, interleaved A/B against lib_r05b.
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
T="tests/test_gpu_octets.py tests/test_gpu_fp32_guard.py tests/test_gpu_kernels.py tests/test_gpu_configs.py"
for v in lib lib_occ2; do
  RRAM_LIB_DIR=$L/$v timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?
  tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests_$v.log | head -30; exit $rc; }
done
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_r05b" - "RRAM_LIB_DIR=$L/lib_occ2" || exit 1
echo done
