#!/bin/bash
# r05x: the C2 line after the per-map statistics refactor (1000 timed maps).
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 400 python bench.py --workload cifar10_quick_mc --steps 10 --warmup 2 > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c2.json')); print(d['value'], d['mc_timed_maps'])"
echo done
