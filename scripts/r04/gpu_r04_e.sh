#!/bin/bash
# Round-4 batch: 1x1 x6 kernel + staged pooling + graph replay + conv1 25-group
# checks, then C5 / graph A/Bs and the conv1 PMC.  Stops at the first failure.
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_kernels.py::test_conv_engine_bf16x6_accuracy_vs_f32 tests/test_gpu_graph.py tests/test_gpu_configs.py tests/test_gpu_kernels.py tests/test_gpu_layers.py tests/test_gpu_wpack.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "err / sum" $O/tests.log | head -30; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL|Error" $O/tests.log | head -40; exit $rc; }
for v in 1 0; do
  timeout -k 10 300 env RRAM_C1X1=$v python -u scripts/gn_layers.py --top 45 > $O/gn_layers_c1x1_$v.txt 2>&1 || { tail -5 $O/gn_layers_c1x1_$v.txt; exit 1; }
  head -1 $O/gn_layers_c1x1_$v.txt
done
for v in 1 0 1 0; do
  timeout -k 10 300 env RRAM_C1X1=$v python bench.py --workload googlenet_sweep --steps 5 --warmup 1 --no-cpu-baseline > $O/c5_$v.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5_$v.json')); print('C5 c1x1=$v', d['value'], d['ms_per_step'], d['roofline'].get('achieved'), d['roofline'].get('engines'))"
done
for w in cifar10_quick_mc lenet_mc cifar10_full_train; do
  for g in 0 1 0 1; do
    timeout -k 10 300 env RRAM_MC_GRAPH=$g python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/${w}_$g.json 2> $O/${w}_$g.err || { tail -5 $O/${w}_$g.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${w}_$g.json')); print('$w graph=$g', d['value'], d['unit'], d['ms_per_step'], d.get('hipgraph'))"
  done
done
REPS=2 bash scripts/ab.sh - || exit 1
mkdir -p gpurun_out/pmcab && KF="conv1|cb" bash scripts/gpu_pmc_ab.sh - || exit 1
grep -E "conv1_ring" gpurun_out/pmcab/v1.txt | cut -c1-700
REPS=2 bash scripts/ab.sh "RRAM_LRN_BLOCKS=4096" "RRAM_LRN_BLOCKS=2048" "RRAM_LRN_BLOCKS=1024" && for v in 1 2 3; do grep -E "pool1|pool2" gpurun_out/ab/v${v}_r2.err | tr "\n" " "; echo; done
