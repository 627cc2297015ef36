#!/bin/bash
# r05y: headline steadiness on one box: the driver's command three times and a
# 200-map run (clock ramp and sustained rate).
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/b20_$r.json 2> $O/b20_$r.err || { tail -5 $O/b20_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b20_$r.json')); print('steps 20', d['value'], d['ms_per_step'])"
done
timeout -k 10 600 python bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/b200.json 2> $O/b200.err || { tail -5 $O/b200.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b200.json')); print('steps 200', d['value'], d['ms_per_step'])"
echo done
