#!/bin/bash
# r05z: MC injection kernel loop: the refactored one-chunk loop (this tree),
# two chunks' loads in flight per trip (lib_ipair) vs the r05 kernel
# (lib_iold): injection bit-exactness tests, kernel-trace averages, headline A/B.
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
for v in lib lib_ipair; do
  RRAM_LIB_DIR=$L/$v timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -k "inject or c2 or c5 or mc" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?
  tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests_$v.log | head -30; exit $rc; }
done
for v in lib_iold lib lib_ipair; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$v -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/kt_$v.log 2>&1 ) || exit 1
  grep -h "k_inject_batched" $O/kt_$v/run_kernel_stats.csv | cut -d, -f1,3,4 | cut -c1-160
done
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_iold" - "RRAM_LIB_DIR=$L/lib_ipair" || exit 1
echo done
