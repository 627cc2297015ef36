#!/bin/bash
# r06n: the TEST-phase head fold (SoftmaxWithLoss + Accuracy over the same scores as one launch,
# rram_softmax_loss_accuracy_fwd); layer / config / graph / MC tests first, then the headline's kernel
# trace (head kernels) and an interleaved A/B against lib_nohead (RRAM_HEAD_FOLD=0).
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_layers.py \
  tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_host.py tests/test_gpu_kernels.py \
  tests/test_gpu_ref_kats.py tests/test_gpu_native_dp.py > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/bench.json 2> $R/$O/bench.err ) || exit 1
grep -i "softmax\|accuracy" $O/prof/*kernel_stats.csv | cut -c1-160
L=$PWD/rram-caffe-simulation_amd
REPS=3 bash scripts/ab.sh - "RRAM_LIB_DIR=$L/lib_nohead" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
