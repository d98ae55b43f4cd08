#!/bin/bash
# Round 3: per-kernel times of the T = 600 match on long/mixed files -- pruned + deferred
# postings pass against the postings kernels alone (one rocprofv3 kernel trace each).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n_pruned -o run --output-format csv -- \
  python3 -u tools/exp/prune_ab.py --profiles 1 --reps 1 route > gpurun_out/r3n_pruned.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n_post -o run --output-format csv -- \
  python3 -u tools/exp/prune_ab.py --profiles 1 --reps 1 off:DICE_PRUNE_WF_ROUTE=0 > gpurun_out/r3n_post.log 2>&1 || exit 3
for d in r3n_pruned r3n_post; do
  echo "== $d"; grep -v "^\[" gpurun_out/$d.log | grep profile
  f=$(find gpurun_out/$d -name "*kernel_stats.csv" | sort | tail -1)
  cut -d, -f1-6 "$f" | head -8
done
