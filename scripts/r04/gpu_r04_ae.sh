#!/bin/bash
# conv backward: data gradient forked onto an auxiliary stream (RRAM_BWD_OVERLAP), A/B on the training configs
set -o pipefail
O=gpurun_out/r04ae; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_solver_kat.py tests/test_gpu_host.py tests/test_gpu_parallel.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_k.log 2>&1; rc=$?
tail -2 $O/tests_k.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests_k.log | head -40; exit $rc; }
for rep in 1 2; do
for ov in 1 0; do
for w in cifar10_full_train lenet_train; do
  RRAM_BWD_OVERLAP=$ov timeout -k 10 300 python bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline > $O/$w.$ov.json 2> $O/$w.$ov.err || { tail -5 $O/$w.$ov.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.$ov.json')); print('overlap=$ov $w', d['value'], d['ms_per_step'])"
done; done; done
RRAM_MC_GRAPH=1 timeout -k 10 300 python bench.py --workload cifar10_full_train --steps 30 --warmup 5 --no-cpu-baseline > $O/graph.json 2> $O/graph.err || { tail -5 $O/graph.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/graph.json')); print('graph', d['value'], d['ms_per_step'], d.get('hipgraph'))"
