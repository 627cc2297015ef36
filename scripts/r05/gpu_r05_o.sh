#!/bin/bash
# r05o: LRN + max pool stores: the octet companion written as consecutive
# 16-byte pieces per lane (this tree) and additionally the pooled y with the
# nontemporal store policy (lib_ynt) vs the r05 kernel storing 48 bytes per
# lane (lib_prev): bit-identity tests, kernel time per variant, headline A/B.
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
for v in lib lib_ynt; do
  RRAM_LIB_DIR=$L/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_octets.py tests/test_gpu_fp32_guard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?
  tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests_$v.log | head -30; exit $rc; }
done
for v in lib_prev lib lib_ynt; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$v -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/kt_$v.log 2>&1 ) || exit 1
  python3 scripts/r05/lrn_stats.py $O/kt_$v $v || exit 1
done
REPS=2 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_prev" - "RRAM_LIB_DIR=$L/lib_ynt" || exit 1
echo done
