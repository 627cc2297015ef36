#!/bin/bash
# r05l: LRN + max pool band kernel with the static register ring and the
# straight-line walk of 32-channel chunks (this tree), with the alternating
# channel direction per chunk (lib_lalt) and without the XCD tile remap
# (lib_lnox): bit-identity tests (b256 planes included) on this tree and
# lib_lalt, kernel time per variant (kernel trace), fetched bytes (FETCH_SIZE).
set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
for v in lib lib_lalt; do
  RRAM_LIB_DIR=$L/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_octets.py -k lrn -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?
  tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests_$v.log | head -30; exit $rc; }
done
for v in lib lib_lalt lib_lnox lib; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$v -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/kt_$v.log 2>&1 ) || exit 1
  python3 scripts/r05/lrn_stats.py $O/kt_$v $v || exit 1
done
for v in lib lib_lalt lib_lnox; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_${v}_FETCH_SIZE -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc_${v}_FETCH_SIZE.log 2>&1 ) || exit 1
  python3 scripts/r05/lrn_stats.py $O/pmc_${v}_FETCH_SIZE $v || exit 1
done
echo done
