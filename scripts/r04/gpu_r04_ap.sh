#!/bin/bash
# kernel sequence per C4 iteration / C2 map after the round-4 launch-count changes
set -o pipefail
O=gpurun_out/r04ap; mkdir -p $O
R=$GRAFT_REPO_ROOT
for w in cifar10_full_train cifar10_quick_mc; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$w -o run -- python3 $R/bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $R/$O/$w.json 2> $R/$O/$w.err) || { tail -5 $O/$w.err; exit 1; }
done
