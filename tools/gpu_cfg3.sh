#!/bin/bash
# Config-3 timing on the GPU box: bench --config 3 (postings kernel by default), REPS runs,
# plus a parity spot check; optional env passes through (e.g. DICE_POST_DENSE=12).
#   bash tools/gpu_cfg3.sh <tag> [reps]
set -u
TAG=$1; REPS=${2:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 3 --extra-configs= --no-cpu-baseline > gpurun_out/${TAG}_$r.json 2> gpurun_out/${TAG}_$r.err || exit 10
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],3), 'ms', '%.4g' % d['value'], d['parity'])" gpurun_out/${TAG}_$r.json
done
