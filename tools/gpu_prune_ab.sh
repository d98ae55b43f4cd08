#!/bin/bash
# Bound-pruned match kernel (dice_prune.hip): its GPU tests, then config-3 bench lines for each
# variant, interleaved over reps. A variant is a comma-separated env list ("base" = defaults).
#   bash tools/gpu_prune_ab.sh <reps> <variant> [variant ...]
#   e.g. bash tools/gpu_prune_ab.sh 2 DICE_POST_PRUNE=0 base DICE_PRUNE_GROUPS=8
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=$1; shift
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/prune_tests.log 2>&1
rc=$?; echo "prune_tests_rc=$rc"; tail -3 gpurun_out/prune_tests.log; [ $rc -eq 0 ] || exit $rc
for r in $(seq 1 $REPS); do
  for v in "$@"; do
    tag=$(echo "$v" | tr -c 'A-Za-z0-9\n' '_')
    envs=$(echo "$v" | tr ',' ' '); [ "$v" = base ] && envs="DICE_NOTHING=1"
    env $envs timeout -k 10 300 python bench.py --config 3 --extra-configs= --no-cpu-baseline --steps 20 --warmup 3 \
      > gpurun_out/ab_${tag}_r$r.json 2> gpurun_out/ab_${tag}_r$r.err || exit 3
    python -c "import json;d=json.load(open('gpurun_out/ab_${tag}_r$r.json'));print('$v r$r', round(d['roofline']['launch_ms'],4), 'ms')"
  done
done
