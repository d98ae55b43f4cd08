#!/bin/bash
# The driver's multi-GPU launch shape at world size 1 (torch.distributed.run, RCCL init,
# barrier/all_reduce timing and the RCCL all_gather of the results).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 2 > gpurun_out/dist1.json 2> gpurun_out/dist1.err || { tail -20 gpurun_out/dist1.err; exit 1; }
cat gpurun_out/dist1.json
