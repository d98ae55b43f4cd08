#!/bin/bash
# Round 3: big-file deferral (coarse-bound files deferred before any exact score): pruned tests,
# A/B against DICE_PRUNE_BIG_DEFER=0 on config-3 and long/mixed files, and the per-phase clocks of
# the pruned kernel (a -DPRUNE3_DIAG=8 build: licensee_amd/lib/var/pdiag8.so); the deferred pass's
# balanced tiles against the previous dice_post.hip (licensee_amd/lib/var/post_prev.so).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_prune.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_g.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/t_g.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/exp/prune_ab.py --reps 3 --profiles 0,1 bigdefer nobig:DICE_PRUNE_BIG_DEFER=0 \
  > gpurun_out/r3g_prune_ab.log 2>&1 || exit 7
grep -v "^\[" gpurun_out/r3g_prune_ab.log
LICENSEE_DICE_LIB=licensee_amd/lib/var/post_prev.so timeout -k 10 600 python -u tools/exp/prune_ab.py --reps 3 --profiles 0,1 prevtiles \
  > gpurun_out/r3g_prev.log 2>&1 || exit 9
grep -v "^\[" gpurun_out/r3g_prev.log
LICENSEE_DICE_LIB=licensee_amd/lib/var/pdiag8.so timeout -k 10 300 python -u tools/exp/prune_ab.py --reps 1 --launches 2 --profiles 0,1 diag \
  > gpurun_out/r3g_phases.log 2>&1 || exit 8
grep -E "phases|profile" gpurun_out/r3g_phases.log | tail -12
