#!/bin/bash
# One GPU-box session: parity tests, smoke, the default bench line (with the CPU
# baseline), a rocprofv3 kernel-trace summary of the same bench command, PMC
# counter passes and an injection grid sweep.  Every GPU step has its own time
# limit; the chain stops at the first failure.  Outputs: gpurun_out/.
#   SKIP_TESTS=1  skip pytest;  PMC=0  skip the counter passes;  SWEEP=0  skip the sweep
set -o pipefail
O=gpurun_out
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/bench_layers.json 2> $O/bench_layers.txt || exit 1
R=$GRAFT_REPO_ROOT
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err ) || { echo "rocprof failed"; tail -20 $O/prof.err; exit 1; }
if [ "${PMC:-1}" = 1 ]; then
  bash scripts/pmc.sh $O/pmc || exit 1
  python scripts/pmc_summary.py $O/pmc > $O/pmc_summary.txt || exit 1
fi
if [ "${SWEEP:-1}" = 1 ]; then
  for g in 2048 8192 1073741824; do
    RRAM_INJECT_GRID=$g timeout -k 10 120 python scripts/kbench.py --only inject > $O/kb_inject_$g.log 2>&1 || exit 1
  done
  timeout -k 10 180 python scripts/kbench.py --only gemm > $O/kb_gemm.log 2>&1 || exit 1
fi
echo session done
