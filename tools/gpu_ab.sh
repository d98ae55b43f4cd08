#!/bin/bash
# Interleaved A/B on one box: every arm runs the same bench.py workload, rep by rep.
#   bash tools/gpu_ab.sh <reps> "<bench args>" <arm> [arm ...]
# An arm is `base` (defaults) or a comma-separated list of `lib:<name>` (licensee_amd/lib/var/<name>.so
# from tools/build_variant.sh) and env settings (`lib:nospill,DICE_POST_PRUNE=0`).
#   e.g. bash tools/gpu_ab.sh 3 "--config 5-T600 --steps 10" base lib:nospill
#        bash tools/gpu_ab.sh 2 "--config 3 --steps 20" base DICE_PRUNE_ROUTE=32
# Prints one line per (rep, arm): launch time, roofline fraction, deferred files (config 3).
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
REPS=$1; ARGS=$2; shift 2
for r in $(seq 1 "$REPS"); do
  for arm in "$@"; do
    tag=$(echo "$arm" | tr -c 'A-Za-z0-9\n' '_')
    envs="DICE_AB_ARM=$tag"
    if [ "$arm" != base ]; then
      for item in $(echo "$arm" | tr ',' ' '); do
        case "$item" in
          lib:*) envs="$envs LICENSEE_DICE_LIB=licensee_amd/lib/var/${item#lib:}.so" ;;
          *) envs="$envs $item" ;;
        esac
      done
    fi
    out=gpurun_out/ab/${tag}_r$r
    env $envs timeout -k 10 300 python bench.py $ARGS --warmup 2 --extra-configs= --no-cpu-baseline --no-extras \
      > $out.json 2> $out.err || { echo "$arm r$r failed (rc $?)"; exit 3; }
    python -c "import json;d=json.load(open('$out.json'));r=d['roofline'];print('$arm r$r', round(r['launch_ms'],4), 'ms frac', round(r['frac'],3), 'parity', d.get('parity'))"
  done
done
