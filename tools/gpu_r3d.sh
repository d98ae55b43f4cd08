#!/bin/bash
# Round 3: full GPU suite + smoke on the padded matrix rows and route 16; the 5-T600 profile
# (PMC: traffic with 128-byte-line rows); routing-point A/B of the pruned match.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 5
echo smoke_ok
bash tools/profile_round.sh r3d_config5_T600 --config 5-T600 || exit 6
timeout -k 10 600 python -u tools/exp/prune_ab.py --reps 3 --profiles 0,1 r16 ra1:DICE_PRUNE_ROUTE_AT=1 \
  ra1r32:DICE_PRUNE_ROUTE_AT=1,DICE_PRUNE_ROUTE=32 r8:DICE_PRUNE_ROUTE=8 > gpurun_out/r3d_prune_ab.log 2>&1 || exit 7
grep -v "^\[" gpurun_out/r3d_prune_ab.log
