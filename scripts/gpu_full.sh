#!/bin/bash
# Round verification on one box: the whole GPU suite, smoke, the headline bench
# line (with the CPU baseline) and a rocprofv3 kernel-trace summary of the same
# bench command.  Each GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
O=gpurun_out; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cat $O/smoke.log | tail -1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err || exit $?
echo done
