#!/bin/bash
# PMC of the 1x1 kernels (GoogLeNet C5 forward).
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
R=$GRAFT_REPO_ROOT
KFILTER=conv1x1 bash scripts/pmc_kernel.sh $O/pmc -- python3 $R/scripts/gn_layers.py --maps 2 > $O/pmc.txt 2>&1 || { tail -5 $O/pmc.txt; exit 1; }
python3 scripts/pmc_clock.py $O/pmc.txt | grep -E "conv1x1" | head -30
grep -E "conv1x1" $O/pmc.txt | cut -c1-700 | head -12
