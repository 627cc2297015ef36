#!/bin/bash
# r05b: octet-kernel patch segment shifts (LDS bank conflicts of conv3/4/5):
# GPU suite, A/B against the round-4 build, LDS conflict counters of this tree.
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$R/rram-caffe-simulation_amd/lib_base" - || exit 1
for v in base new; do
  L=$R/rram-caffe-simulation_amd/lib; [ $v = base ] && L=$R/rram-caffe-simulation_amd/lib_base
  ( cd /tmp && export TMPDIR=/tmp && RRAM_LIB_DIR=$L timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/$O/pmc_$v -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc_$v.log 2>&1 ) || exit 1
done
echo done
