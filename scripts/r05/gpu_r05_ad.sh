#!/bin/bash
# r05ad: overlapped injection (the default now) vs serial (RRAM_MC_OVERLAP=0)
# on the live bench (no --profile-layers: the layer table comes from maps
# after the timed region), 20 and 200 maps, interleaved.
set -o pipefail
PROFILE_FLAG= REPS=4 scripts/ab.sh - "RRAM_MC_OVERLAP=0" || exit 1
PROFILE_FLAG= STEPS=200 REPS=2 scripts/ab.sh - "RRAM_MC_OVERLAP=0" || exit 1
echo done
