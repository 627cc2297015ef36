#!/bin/bash
# Try a kernel variant on one box: the GPU tests named in $TESTS under the
# environment $TENV (default: the octet / conv / guard files), then the
# interleaved bench A/B of the variants given as arguments (scripts/ab.sh).
#   scripts/gpu_try.sh "RRAM_LIB_DIR=rram-caffe-simulation_amd/lib_base" -   (baseline build vs this tree)
set -o pipefail
O=gpurun_out/try; mkdir -p $O
T=${TESTS:-tests/test_gpu_octets.py tests/test_gpu_wpack.py tests/test_gpu_fp32_guard.py tests/test_gpu_kernels.py}
timeout -k 10 900 env ${TENV:-} python -u -m pytest $T -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "err / sum" $O/tests.log; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
[ $# -gt 0 ] && REPS=${REPS:-3} scripts/ab.sh "$@"
