#!/bin/bash
# Bound-pruned match kernel (dice_prune.hip): its GPU tests, then config-3 bench lines for the
# postings kernel (DICE_POST_PRUNE=0) and each pruned schedule (DICE_PRUNE_SCHED), interleaved.
#   bash tools/gpu_prune_ab.sh [reps]
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${1:-2}
timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/prune_tests.log 2>&1
rc=$?; echo "prune_tests_rc=$rc"; tail -3 gpurun_out/prune_tests.log; [ $rc -eq 0 ] || exit $rc
for r in $(seq 1 $REPS); do
  for v in post s0 s1 s2; do
    if [ $v = post ]; then env="DICE_POST_PRUNE=0"; else env="DICE_PRUNE_SCHED=${v#s}"; fi
    env $env timeout -k 10 300 python bench.py --config 3 --extra-configs= --no-cpu-baseline --steps 20 --warmup 3 \
      > gpurun_out/prune_${v}_r$r.json 2> gpurun_out/prune_${v}_r$r.err || exit 3
    echo "$v r$r $(python -c "import json;d=json.load(open('gpurun_out/prune_${v}_r$r.json'));print(d['ms_per_step'], d['roofline']['launch_ms'] if 'launch_ms' in d['roofline'] else '', d.get('parity',{}).get('mismatches'))")"
  done
done
