#!/bin/bash
# kernel sequence per map / iteration of the launch-bound configs (C2 CIFAR-10 quick MC, C1 LeNet MC, C5 GoogLeNet)
set -o pipefail
O=gpurun_out/r04aa; mkdir -p $O
R=$GRAFT_REPO_ROOT
for w in cifar10_quick_mc lenet_mc; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$w -o run -- python3 $R/bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/$w.json 2> $R/$O/$w.err) || { tail -5 $O/$w.err; exit 1; }
done
for w in cifar10_quick_mc lenet_mc; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/b_$w.json 2> $O/b_$w.err || { tail -5 $O/b_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$w.json')); print('$w', d['value'], d['ms_per_step'])"
done
