#!/bin/bash
# r05s: the pooled-output fold (this tree: a folded LRN + max pool whose top
# only a convolution reads writes only the octet companion; the fp32 top is
# materialised on read) vs the same tree without it (lib_nofold): the whole
# GPU suite on this tree, LRN kernel times, interleaved headline A/B.
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/pytest_gpu.log | head -30; exit $rc; }
for v in lib_nofold lib; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$v -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/kt_$v.log 2>&1 ) || exit 1
  python3 scripts/r05/lrn_stats.py $O/kt_$v $v || exit 1
done
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_nofold" - || exit 1
echo done
