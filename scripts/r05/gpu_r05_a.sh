#!/bin/bash
# r05a: conv2/conv5 k_conv_cb16_x6 per-parity instantiations (no scratch) +
# knob pruning: full GPU suite, then an interleaved A/B against the round-4
# build (lib_base), the kernel trace and the traffic passes of this tree.
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" $O/tests.log | head -30; exit $rc; }
REPS=3 scripts/ab.sh "RRAM_LIB_DIR=$R/rram-caffe-simulation_amd/lib_base" - || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err ) || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $R/$O/pmc_$c -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/pmc_$c.log 2>&1 ) || exit 1
done
echo done
