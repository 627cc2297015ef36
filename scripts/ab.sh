#!/bin/bash
# One parameterised A/B driver for the headline bench: each argument is one
# variant, a space-separated list of environment assignments ("-" = none);
# the variants run alternately ${REPS:-2} times (bench --profile-layers unless
# PROFILE_FLAG is set, e.g. PROFILE_FLAG= for the live bench,
# ${STEPS:-20} steps), one summary line per run.  Extra bench flags: $BENCH_ARGS.
#   scripts/ab.sh - "RRAM_MC_OVERLAP=0" "RRAM_LIB_DIR=$PWD/rram-caffe-simulation_amd/lib_x"
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=(); [ "$v" != "-" ] && read -ra envs <<< "$v"
    timeout -k 10 300 env "${envs[@]}" python bench.py --no-cpu-baseline ${PROFILE_FLAG---profile-layers} --steps ${STEPS:-20} ${BENCH_ARGS:-} \
      > $O/v${i}_r$r.json 2> $O/v${i}_r$r.err || { tail -5 $O/v${i}_r$r.err; exit 1; }
    python3 - "$O/v${i}_r$r.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
L = d["roofline"]["contractions"]["layers"]
print(f"[{sys.argv[2]}] {d['value']:.0f} img/s  {d['ms_per_step']:.3f} ms/step  inject {d['roofline_inject']['avg_us_per_launch']:.0f} us  "
      + " ".join(f"{k} {v['ms']:.3f}" for k, v in L.items()), flush=True)
PY
  done
done
