#!/bin/bash
# r05q: LRN + max pool with odd channel chunks walking down (lib_lalt: the
# halo channels two chunks share are read at the same time, so the second
# read can hit L2) vs this tree, now that the kernel streams ~5 TB/s:
# bit-identity tests on lib_lalt, kernel time (two traces each, interleaved).
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
RRAM_LIB_DIR=$L/lib_lalt timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_octets.py -k "lrn or pool" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_lib.log 2>&1; rc=$?
tail -1 $O/tests_lib.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests_lib.log | head -30; exit $rc; }
for r in 1 2; do for v in lib_lalt lib; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_${v}_$r -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/kt_${v}_$r.log 2>&1 ) || exit 1
  python3 scripts/r05/lrn_stats.py $O/kt_${v}_$r $v || exit 1
done; done
echo done
