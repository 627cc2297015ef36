#!/bin/bash
# conv1 PMC + GoogLeNet kernel-trace profile
set -o pipefail
O=gpurun_out; mkdir -p $O
R=$GRAFT_REPO_ROOT
KFILTER=conv1 timeout -k 10 400 scripts/pmc_kernel.sh $O/pmc_c1 -- python3 $R/scripts/conv1_check.py --iters 3 > $O/pmc_c1.txt 2>&1 || { cat $O/pmc_c1.txt; exit 1; }
cat $O/pmc_c1.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_gn -o run --output-format csv -- python3 $R/bench.py --workload googlenet_sweep --steps 2 --warmup 1 > $R/$O/gn_bench.json 2> $R/$O/gn_bench.err || { tail $R/$O/gn_bench.err; exit 1; }
cat $R/$O/gn_bench.json
head -30 $R/$O/prof_gn/*/run_kernel_stats.csv
