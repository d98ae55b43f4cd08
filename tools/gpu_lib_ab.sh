#!/bin/bash
# Interleaved A/B of library builds (tools/build_variant.sh) on the config-3 pruned match:
#   tools/gpu_lib_ab.sh <reps> <name>...   (name "base" = licensee_amd/lib/liblicensee_dice.so)
export TMPDIR=/tmp
REPS=$1; shift
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    if [ "$v" = base ]; then unset LICENSEE_DICE_LIB; else export LICENSEE_DICE_LIB=licensee_amd/lib/var/$v.so; fi
    timeout -k 10 240 python -u tools/exp/prune_ab.py --reps 1 --profiles ${PROFILES:-0} v3 2>&1 | grep " ms " | sed "s/^/$v rep$rep: /" || exit 1
  done
done
