#!/bin/bash
# Round 3: matrix kernel with uniform row bases (no spilled store addresses): matrix parity tests,
# A/B against the previous dice_post.hip on config 5-T600, the torchrun world-size-1 bench check.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_h.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/t_h.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_matrix_ab.sh 2 base post_prev || exit 2
bash tools/gpu_dist_check.sh > gpurun_out/dist_check.log 2>&1 || { tail -5 gpurun_out/dist_check.log; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/dist1.json'));print('torchrun ws1', d['value'], d['n_gpus'], d['extras'].get('gather_winner'), d['extras'].get('rccl_allgather_ms'), d['extras'].get('host_gather_ms'))"
