#!/bin/bash
# conv2 traffic: 16x16x32 (default) vs 32x32 octet kernel (RRAM_CB16=4), PMC passes.
set -o pipefail
mkdir -p gpurun_out/pmcab
KF="cb" bash scripts/gpu_pmc_ab.sh - "RRAM_CB16=4" 2>&1 | grep -v "declare -x" || exit 1
for v in 1 2; do grep -E "conv_cb" gpurun_out/pmcab/v$v.txt | grep -E "grid=   786432|grid=   173056" | sed -E 's/SQ_WAVE.*(FETCH_SIZE=[^ ]+ WRITE_SIZE=[^ ]+).*/\1/'; done
