#!/bin/bash
# PMC passes only (scripts/pmc.sh) over the default bench, summary per kernel.
set -o pipefail
TAG=${1:-pmc}
timeout -k 10 900 bash scripts/pmc.sh gpurun_out/$TAG || exit $?
python3 scripts/pmc_summary.py gpurun_out/$TAG > gpurun_out/$TAG/summary.txt && python3 scripts/pmc_traffic.py gpurun_out/$TAG > gpurun_out/$TAG/traffic.json
head -8 gpurun_out/$TAG/summary.txt | cut -c1-400
