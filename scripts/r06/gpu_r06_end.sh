#!/bin/bash
# r06end: the full GPU suite, smoke and the headline bench line on the final tree.
set -o pipefail
O=gpurun_out/r06end; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 400 python bench.py --workload googlenet_sweep --steps 10 --warmup 2 --no-cpu-baseline > $O/gn.json 2> $O/gn.err || exit 1
python3 -c "
import json; d=json.loads(open('$O/gn.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
