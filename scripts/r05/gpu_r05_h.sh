#!/bin/bash
# r05h: conv1 on k_conv1_pair_x6 (two workgroups of six waves per CU) -- lib --
# vs the ring kernel (lib_c1ring, -DRRAM_C1_RING): GPU suite on lib, headline
# A/B, kernel traces of one C4 training run on lib and lib_occ2 (the
# gathered weight gradient vs im2col + GEMM).
set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_c1ring" - || exit 1
# fc6 / fc7 k_gemm_x6 DMA ablations (diagnostic builds, wrong results: layer times only)
REPS=1 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_fca1" "RRAM_LIB_DIR=$L/lib_fca2" - || exit 1
for v in lib lib_occ2 lib_im2t2; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c4_$v -o run --output-format csv -- python3 $R/bench.py --workload cifar10_full_train --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/c4_$v.json 2> $R/$O/c4_$v.err ) || exit 1
done
for r in 1 2; do for v in lib_occ2 lib lib_im2t2; do
  RRAM_LIB_DIR=$L/$v timeout -k 10 300 python bench.py --workload cifar10_full_train --steps 20 --warmup 3 --no-cpu-baseline > $O/c4b_$v.json 2> $O/c4b_$v.err || { tail -5 $O/c4b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4b_$v.json')); print('C4 $v', d['value'], d['ms_per_step'])"
done; done
echo done
