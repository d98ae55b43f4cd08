#!/bin/bash
# Fused vs split postings kernels on config 3 (parity under DICE_POST_FUSED=1, then timings).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
DICE_POST_FUSED=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_corpus_sizes.py tests/test_gpu_slowpath.py -m gpu -x -q -k "post or config3" --timeout 300 --timeout-method thread > gpurun_out/t_fused.log 2>&1
rc=$?; echo "fused_tests_rc=$rc"; tail -3 gpurun_out/t_fused.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do DICE_POST_FUSED=$v bash tools/gpu_cfg3.sh c3fused$v 1 || exit 9; done
for g in ${FUSED_DIAG:-1 2 8}; do DICE_POST_FUSED=1 DICE_POST_DIAG=$g bash tools/gpu_cfg3.sh c3fdiag$g 1 || exit 9; done
