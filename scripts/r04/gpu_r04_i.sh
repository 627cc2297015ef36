#!/bin/bash
# PMC of the IP / conv kernels of the headline bench (all kernels listed).
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
R=$GRAFT_REPO_ROOT
bash scripts/pmc_kernel.sh $O/pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc.txt 2>&1 || { tail -5 $O/pmc.txt; exit 1; }
grep -E "gemm_x6|splitk|gemm<|conv_cb|conv1_ring|pack" $O/pmc.txt | cut -c1-900
