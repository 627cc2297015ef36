#!/bin/bash
# fc6 / fc7 tile A/B: 256 x 128 (default) vs 128 x 256 (RRAM_GX6_T128=1).
set -o pipefail
REPS=3 bash scripts/ab.sh - "RRAM_GX6_T128=1" || exit 1
