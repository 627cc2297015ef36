#!/bin/bash
# r05t: split-K GEMMs with M <= 32 (the CIFAR-10 / LeNet weight gradients) on
# 32 x 128 tiles (this tree) vs 64 x 64 (lib_thin0): conv / IP backward and
# C4 / LeNet training tests, the C4 iteration's kernel trace per variant,
# interleaved C4 / LeNet training A/B.
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_solver_kat.py tests/test_gpu_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
for v in lib_thin0 lib; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c4_$v -o run --output-format csv -- python3 $R/bench.py --workload cifar10_full_train --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/c4_$v.json 2> $R/$O/c4_$v.err ) || exit 1
  python3 scripts/kernel_sequence.py $O/c4_$v $v > $O/c4_seq_$v.txt || exit 1
  head -1 $O/c4_seq_$v.txt
done
for r in 1 2 3; do for v in lib_thin0 lib; do
  for w in cifar10_full_train lenet_train; do
    RRAM_LIB_DIR=$L/$v timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/${w}_${v}_$r.json 2> $O/${w}_${v}_$r.err || { tail -5 $O/${w}_${v}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/${w}_${v}_$r.json "$w $v"
  done
done; done
echo done
