#!/bin/bash
# PMC passes (each its own rocprofv3 run) over one developer command; prints
# per-kernel counter sums for kernels matching $KFILTER.
#   usage: KFILTER=conv1_ring scripts/pmc_kernel.sh OUTDIR -- python3 scripts/conv1_check.py
set -o pipefail
OUT=$1; shift; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/p$i -o run -- "$@" > $R/$OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $R/$OUT/p$i.log; exit 1; }
done
cd $R && python3 scripts/pmc_summary.py $OUT
