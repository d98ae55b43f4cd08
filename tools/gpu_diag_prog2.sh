#!/bin/bash
# Sparse-program diagnostic builds on config 2 (results wrong): full / no accumulate / no epilogue.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in full noacc noepi full noacc; do
  e=""; [ $v != full ] && e="DICE_PROG_DIAG=$v"
  env $e timeout -k 10 300 python bench.py --steps 50 --warmup 5 --extra-configs= --no-cpu-baseline > gpurun_out/dg_$v.json 2> gpurun_out/dg_$v.err || exit 10
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['roofline']['launch_ms']*1e3,2), 'us')" gpurun_out/dg_$v.json
done
