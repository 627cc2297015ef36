#!/bin/bash
# SQ/GRBM counter passes over a short bench.py run for each RRAM_GEMM_V2
# setting (k_gemm2 vs k_gemm), summarised per kernel: scripts/gpu_pmc_ab.sh TAG "3 0"
set -o pipefail
TAG=${1:-pmcab}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${2:-3 0}; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    env RRAM_${ABVAR:-GEMM_V2}=$v timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/v$v/p$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/v$v.p$i.log 2>&1 || { echo "v$v pass $i failed"; tail -5 $O/v$v.p$i.log; exit 1; }
  done
  python3 $R/scripts/pmc_summary.py $O/v$v > $O/v$v.txt
done
echo done
