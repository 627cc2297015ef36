#!/bin/bash
# r05k: LRN + max pool band kernel variants vs this tree: alternating channel
# walk direction per chunk (lib_lalt), no XCD tile remap (lib_lnox), 2048-block
# grid target (lib_lb2k): bit-identity tests on the alternating walk, kernel
# time per variant (kernel trace) and fetched bytes (FETCH_SIZE pass).
set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
RRAM_LIB_DIR=$L/lib_lalt timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_octets.py -k lrn -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_lalt.log 2>&1; rc=$?
tail -1 $O/tests_lalt.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests_lalt.log | head -30; exit $rc; }
for v in lib lib_lalt lib_lnox lib_lb2k lib; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$v -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/kt_$v.log 2>&1 ) || exit 1
  python3 scripts/r05/lrn_stats.py $O/kt_$v $v || exit 1
done
for v in lib lib_lalt lib_lnox lib_lb2k; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_${v}_FETCH_SIZE -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc_${v}_FETCH_SIZE.log 2>&1 ) || exit 1
  python3 scripts/r05/lrn_stats.py $O/pmc_${v}_FETCH_SIZE $v || exit 1
done
echo done
