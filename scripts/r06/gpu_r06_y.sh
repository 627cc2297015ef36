#!/bin/bash
# r06y: PMC passes (scripts/pmc_kernel.sh) over the GoogLeNet sweep workload: per-kernel MFMA busy, waits,
# LDS conflicts, clock and HBM bytes of the 1x1 / 3x3 / pool kernels.
set -o pipefail
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 800 bash scripts/pmc_kernel.sh $O/pmc -- python3 $GRAFT_REPO_ROOT/bench.py --workload googlenet_sweep \
  --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc.txt 2>&1; rc=$?
tail -40 $O/pmc.txt | cut -c1-400; exit $rc
