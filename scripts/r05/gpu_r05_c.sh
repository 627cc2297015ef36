#!/bin/bash
# r05c: octet-kernel segment shifts (lib_r05b) and + the 2-ahead weight ring of
# the 3x3 32x32 octet kernel (lib): GPU suite on this tree, interleaved A/B of
# round-4 / r05b / this tree, LDS conflict and instruction-cache counters.
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
R=$GRAFT_REPO_ROOT
L=$R/rram-caffe-simulation_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$L/lib_base" "RRAM_LIB_DIR=$L/lib_r05b" - || exit 1
for v in lib_base lib; do
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L/$v timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $R/$O/pmc_lds_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc_lds_$v.log 2>&1 ) || exit 1
done
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $R/$O/pmc_ic -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc_ic.log 2>&1 ) || exit 1
echo done
