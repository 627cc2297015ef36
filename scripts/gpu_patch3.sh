#!/bin/bash
# full GPU suite + bench x2 at the current default policy
set -o pipefail
O=gpurun_out/patch3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 python scripts/kbench.py --only gemm > $O/kb.txt 2>&1 || exit 1
for r in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline --profile-layers > $O/b_$r.json 2> $O/b_$r.err || exit 1; done
echo done
