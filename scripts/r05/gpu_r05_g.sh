#!/bin/bash
# r05g: (1) octet-kernel plans at two workgroups per CU (conv3 128x128, conv4 /
# conv5 64x128) and (2) the weight gradient gathered inside its GEMM (IM2T,
# no im2col) -- lib -- against r05d's lib_occ2; (3) fc6/fc7 on the 8-wave
# k_gemm_x6 (lib_fcnw8); (4) C4 data gradients always as a flipped-kernel
# forward (lib_dxall).  Full GPU suite on lib, headline A/B, C4 A/B, conv1
# stamp shares (lib_c1stamp).
set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
RRAM_LIB_DIR=$L/lib_fcnw8 timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32_guard.py tests/test_gpu_ref_kats.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_fc.log 2>&1; rc=$?
tail -1 $O/tests_fc.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests_fc.log | head -30; exit $rc; }
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_occ2" - "RRAM_LIB_DIR=$L/lib_fcnw8" || exit 1
for r in 1 2; do for v in lib_occ2 lib lib_dxall; do
  RRAM_LIB_DIR=$L/$v timeout -k 10 300 python bench.py --workload cifar10_full_train --steps 20 --warmup 3 --no-cpu-baseline > $O/c4_$v.json 2> $O/c4_$v.err || { tail -5 $O/c4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_$v.json')); print('C4 $v', d['value'], d['ms_per_step'])"
done; done
RRAM_LIB_DIR=$L/lib_c1stamp timeout -k 10 300 python scripts/c1_stamp.py > $O/c1_stamp.txt 2>&1 || exit 1
cat $O/c1_stamp.txt
echo done
