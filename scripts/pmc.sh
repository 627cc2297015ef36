#!/bin/bash
# PMC counter passes (each its own rocprofv3 run, --pmc only with kernel dispatch
# records; no sys/runtime trace) over a short bench.py run.  Usage: scripts/pmc.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/pmc}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/$OUT/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo pmc done
