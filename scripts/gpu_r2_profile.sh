#!/bin/bash
# One GPU-box session at HEAD: the full GPU parity suite, smoke(), the
# headline bench under rocprofv3 --kernel-trace --stats (so the bench line and
# the kernel summary describe the same run), then the PMC passes of
# scripts/pmc.sh.  Every GPU step has its own time limit; the chain stops at
# the first failure.  Usage: scripts/gpu_r2_profile.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  cat $O/smoke.log
fi
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run \
    --output-format csv -- python3 $R/bench.py > $O/bench_line.json 2> $O/bench.err ) || { echo "bench under rocprof failed"; tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench_line.json
timeout -k 10 900 bash $R/scripts/pmc.sh gpurun_out/$TAG/pmc || exit $?
python3 $R/scripts/pmc_traffic.py $O/pmc > $O/pmc_traffic.json && python3 $R/scripts/pmc_summary.py $O/pmc > $O/pmc_summary.txt
head -12 $O/pmc_summary.txt | cut -c1-260
echo session done
