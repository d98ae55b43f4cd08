#!/bin/bash
# GPU session: torchrun N=1 bench line, then rocprofv3 passes for configs 2, 5, 4, 3.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 > gpurun_out/torchrun1.json 2> gpurun_out/torchrun1.err || exit 11
cut -c1-400 gpurun_out/torchrun1.json
for c in 2 5 4 3; do
  bash tools/profile_round.sh round1b_config$c --config $c || exit $?
  echo "profiled config $c"
done
