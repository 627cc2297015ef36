#!/bin/bash
# GPU check of a kernel change: full GPU parity suite, per-layer bench (twice),
# one LDS PMC pass.  Each GPU step has its own time limit; stops at the first failure.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_ab.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/ab_bench$i.json 2> $O/ab_bench$i.err || exit $?
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/$O/ab_pmc -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/ab_pmc.log 2>&1 || exit $?
echo done
