#!/bin/bash
# r05n: (1) k_conv1_ring_x6 without scratch (refill addresses re-derived per
# use, weight fragments by buffer loads: this tree) and with a 2-group weight
# ring prefetching across the tile boundary (lib_c1r2) vs the r05 HEAD kernel
# (lib_prev, 20 B of scratch, a vmcnt(0) per reload): GPU tests on both new
# builds, interleaved headline A/B; (2) LRN + max pool pooling diagnostics:
# no y store (lib_ld4), no LDS tap reads (lib_ld5), no in-order re-walk
# (lib_ld6), no pooling at all (lib_ld2) -- bounds only, garbage values.
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
T="tests/test_gpu_kernels.py tests/test_gpu_x6_range.py tests/test_gpu_fp32_guard.py"
for v in lib lib_c1r2; do
  RRAM_LIB_DIR=$L/$v timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?
  tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests_$v.log | head -30; exit $rc; }
done
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_prev" - "RRAM_LIB_DIR=$L/lib_c1r2" || exit 1
for v in lib lib_ld2 lib_ld4 lib_ld5 lib_ld6; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$v -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/kt_$v.log 2>&1 ) || exit 1
  python3 scripts/r05/lrn_stats.py $O/kt_$v $v || exit 1
done
echo done
