#!/bin/bash
# GoogLeNet C5: kernel trace (per-kernel durations) + PMC passes of the 1x1 kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04g; mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt -o run -- python3 $R/scripts/gn_layers.py --maps 3 > $R/$O/kt.log 2>&1) || { tail -5 $O/kt.log; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp $f $O/googlenet_kernel_stats.csv; head -40 $O/googlenet_kernel_stats.csv | cut -c1-180
KFILTER=conv1x1 bash scripts/pmc_kernel.sh $O/pmc -- python3 $R/scripts/gn_layers.py --maps 2 > $O/pmc.txt 2>&1 || { tail -5 $O/pmc.txt; exit 1; }
python3 scripts/pmc_clock.py $O/pmc.txt | grep -E "conv1x1|pool|gemm" | head -40
