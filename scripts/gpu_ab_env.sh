#!/bin/bash
# A/B of a tuning knob: per-layer bench with and without the environment
# assignment in $AB (e.g. AB="RRAM_GEMM_TILE=96256"), alternated twice.
set -o pipefail
O=gpurun_out
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers --steps 20 > $O/ab_base$i.json 2> $O/ab_base$i.err || exit $?
  timeout -k 10 300 env $AB python bench.py --no-cpu-baseline --profile-layers --steps 20 > $O/ab_var$i.json 2> $O/ab_var$i.err || exit $?
done
echo done
