#!/bin/bash
# Round 3: the pruned-kernel tests with the 32-group bound, then A/B of 32 vs 16 groups and the
# routing threshold with 32 groups, on config-3 and long/mixed files.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_e.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/t_e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/exp/prune_ab.py --reps 3 --profiles 0,1 ref g16:DICE_PRUNE_GROUPS=16 \
  refr32:DICE_PRUNE_ROUTE=32 refe16:DICE_PRUNE_MAX_EVALS=16 g16e16:DICE_PRUNE_GROUPS=16,DICE_PRUNE_MAX_EVALS=16 > gpurun_out/r3e_prune_ab.log 2>&1 || exit 7
grep -v "^\[" gpurun_out/r3e_prune_ab.log
