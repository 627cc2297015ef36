#!/bin/bash
# r05m: (1) LRN + max pool diagnostics: kernel time with no LRN arithmetic
# (lib_ld1), no pooling (lib_ld2), no barrier (lib_ld3) vs this tree -- bounds
# only, the diagnostic builds compute garbage; (2) the r05j A/B: k_conv_cb16_x6
# with 2-group patch staging distance (lib_sd2) and band-ordered row tiles
# (lib_band, 48 columns per band): octet tests on both, interleaved headline
# A/B, FETCH / WRITE of the band order.
set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
for v in lib lib_ld1 lib_ld2 lib_ld3; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$v -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/kt_$v.log 2>&1 ) || exit 1
  python3 scripts/r05/lrn_stats.py $O/kt_$v $v || exit 1
done
T="tests/test_gpu_octets.py tests/test_gpu_fp32_guard.py"
for v in lib_sd2 lib_band; do
  RRAM_LIB_DIR=$L/$v timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?
  tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests_$v.log | head -30; exit $rc; }
done
REPS=3 scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_sd2" "RRAM_LIB_DIR=$L/lib_band" || exit 1
for v in lib lib_band; do for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $R/$O/pmc_${v}_$c -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc_${v}_$c.log 2>&1 ) || exit 1
done; done
echo done
