#!/bin/bash
# Round-6 record on one box: scripts/gpu_final.sh into $O (GPU suite, smoke, headline line with the CPU
# baseline, kernel trace, PMC passes + traffic table + summary, the other configs' lines, GoogLeNet trace),
# then the C4 training iteration's kernel sequence.
set -o pipefail
export O=${O:-gpurun_out/r06u}
R=$GRAFT_REPO_ROOT
bash scripts/gpu_final.sh || exit $?
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c4 -o run --output-format csv -- python3 $R/bench.py --workload cifar10_full_train --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/c4.json 2> $R/$O/c4.err ) || exit 1
python3 scripts/kernel_sequence.py $O/c4 cifar10_full_train > $O/c4_sequence.txt || exit 1
head -1 $O/c4_sequence.txt
echo final-done
