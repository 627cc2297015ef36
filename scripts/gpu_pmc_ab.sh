#!/bin/bash
# PMC passes of the headline bench under each variant given as an argument
# (space-separated env assignments, "-" = none): per-kernel effective clock,
# MFMA busy and the counter table (scripts/pmc_kernel.sh + pmc_clock.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
i=0
for v in "$@"; do
  i=$((i + 1))
  envs=(); [ "$v" != "-" ] && read -ra envs <<< "$v"
  ( export "${envs[@]}" 2>/dev/null; bash scripts/pmc_kernel.sh gpurun_out/pmcab/v$i -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcab/v$i.txt ) || exit 1
  echo "== [$v]"; python3 scripts/pmc_clock.py gpurun_out/pmcab/v$i.txt | grep -E "${KF:-.}"
done
