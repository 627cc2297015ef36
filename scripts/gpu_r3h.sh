#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --workload googlenet_sweep --steps 10 --warmup 2 > $O/wl_googlenet_sweep.json 2> $O/wl_gn.err || { tail -5 $O/wl_gn.err; exit 1; }
cut -c1-200 $O/wl_googlenet_sweep.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$O/prof_gn -o run --output-format csv -- python3 $R/bench.py --workload googlenet_sweep --steps 2 --warmup 1 --no-cpu-baseline > $R/$O/prof_gn_bench.json 2> $R/$O/prof_gn.err ) || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_h.json 2> $O/bench_h.err || exit $?
cut -c1-200 $O/bench_h.json
