#!/bin/bash
# r06t: k_conv_s2_x6 alone at b256 (time, TFLOP/s) and its PMC counters (MFMA busy, waits, clock, LDS conflicts).
set -o pipefail
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 120 python3 scripts/s2_check.py > $O/s2.json 2> $O/s2.err || { tail -5 $O/s2.err; exit 1; }
cat $O/s2.json
KFILTER=conv_s2 timeout -k 10 600 bash scripts/pmc_kernel.sh $O/pmc -- python3 $GRAFT_REPO_ROOT/scripts/s2_check.py --iters 5 > $O/pmc.txt 2>&1; rc=$?
cat $O/pmc.txt | tail -30; exit $rc
