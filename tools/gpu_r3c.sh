#!/bin/bash
# Round 3: deferral tuning of the pruned match (route threshold after two exact scores, max
# exact scores before deferral) on config-3 files and long/mixed files, in one process.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/exp/prune_ab.py --reps 3 --profiles 0,1 v4 r16:DICE_PRUNE_ROUTE=16 \
  r64:DICE_PRUNE_ROUTE=64 e16:DICE_PRUNE_MAX_EVALS=16 r64e16:DICE_PRUNE_ROUTE=64,DICE_PRUNE_MAX_EVALS=16 \
  r8e4:DICE_PRUNE_ROUTE=8,DICE_PRUNE_MAX_EVALS=4 post:DICE_POST_PRUNE=0 > gpurun_out/r3c_prune_ab.log 2>&1
rc=$?; cat gpurun_out/r3c_prune_ab.log | grep -v "^\[" ; exit $rc
