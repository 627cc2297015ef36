#!/bin/bash
# A/B of the bf16x6 engine: the GPU parity suite, then the bench with
# per-layer times with the engine off (RRAM_X6=0) and on.
set -o pipefail
O=gpurun_out/x6
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head -20; exit $rc; }
grep "bf16x6 .*e-" $O/pytest.log | head -8
AB=${AB:-RRAM_X6}
for x in 0 1; do
  env $AB=$x timeout -k 10 300 python bench.py --no-cpu-baseline --profile-layers > $O/bench_$x.json 2> $O/layers_$x.txt || exit 1
  cut -c1-200 $O/bench_$x.json
done
