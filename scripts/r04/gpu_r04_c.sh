#!/bin/bash
# MC hipGraph replay check + small-config A/B (graph vs eager) + LRN block-target A/B.
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_wpack.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $rc; }
for w in cifar10_quick_mc lenet_mc cifar10_full_train; do
  for g in 0 1 0 1; do
    timeout -k 10 300 env RRAM_MC_GRAPH=$g python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/${w}_$g.json 2> $O/${w}_$g.err || { tail -5 $O/${w}_$g.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${w}_$g.json')); print('$w graph=$g', d['value'], d['unit'], d['ms_per_step'], d.get('hipgraph'))"
  done
done
[ -n "$NO_LRN" ] || { REPS=2 bash scripts/ab.sh "RRAM_LRN_BLOCKS=4096" "RRAM_LRN_BLOCKS=2048" "RRAM_LRN_BLOCKS=1024" && for v in 1 2 3; do grep -E "pool1|pool2" gpurun_out/ab/v${v}_r2.err | tr "\n" " "; echo; done; }
