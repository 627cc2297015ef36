#!/bin/bash
# conv forward split-K target sweep at round-4 end (RRAM_CONV_SPLIT workgroups)
set -o pipefail
O=gpurun_out/r04aq; mkdir -p $O
for rep in 1 2; do for sp in 1024 2048 512; do for w in cifar10_quick_mc cifar10_full_train lenet_mc; do
  RRAM_CONV_SPLIT=$sp timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.json')); print('split=$sp $w', d['value'], d['ms_per_step'])"
done; done; done
