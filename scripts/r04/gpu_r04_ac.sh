#!/bin/bash
# split-K fp32 convolution forward for thin short-grid layers (CIFAR-10 / LeNet), A/B against RRAM_CONV_SPLIT=0
set -o pipefail
O=gpurun_out/r04ac; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_layers.py -m gpu -x -q -k "split or conv or c1 or c2 or c4 or lenet or cifar" --timeout 120 --timeout-method thread > $O/tests_k.log 2>&1; rc=$?
tail -2 $O/tests_k.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_k.log | head -40; exit $rc; }
for rep in 1 2; do
for sp in 0 1; do
for w in cifar10_quick_mc lenet_mc cifar10_full_train lenet_train; do
  RRAM_CONV_SPLIT=$sp timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/$w.$sp.json 2> $O/$w.$sp.err || { tail -5 $O/$w.$sp.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.$sp.json')); print('split=$sp $w', d['value'], d['ms_per_step'])"
done; done; done
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/bench.py --workload cifar10_quick_mc --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/c2p.json 2> $R/$O/c2p.err) || { tail -5 $O/c2p.err; exit 1; }
