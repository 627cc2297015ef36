#!/bin/bash
# Round-4 parity record: the fp32-level guard + reference KATs + changed host
# paths, then the guard against a build with one bf16x6 product term dropped
# (must FAIL: pytest exit 1 expected), then the whole GPU suite and a bench line.
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_fp32_guard.py tests/test_gpu_ref_kats.py tests/test_gpu_wpack.py tests/test_gpu_solver_kat.py -m gpu -s > $O/new.log 2>&1; rc=$?
tail -3 $O/new.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/new.log | head -30; exit $rc; }
for k in ${DROPS:-1}; do
  RRAM_LIB_DIR=$PWD/rram-caffe-simulation_amd/lib_drop$k timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_fp32_guard.py -m gpu -s > $O/drop$k.log 2>&1; rc=$?
  echo "drop $k: pytest rc $rc (1 = guard failed as it must)"; grep -E "err / sum|PASSED|FAILED" $O/drop$k.log | head -20
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/all.log 2>&1; rc=$?
tail -3 $O/all.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/all.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
