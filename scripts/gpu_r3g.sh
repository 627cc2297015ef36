#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python scripts/x6_range_probe.py > $O/x6_range.txt 2>&1 || { tail -20 $O/x6_range.txt; exit 1; }
./scripts/gpu_full.sh
