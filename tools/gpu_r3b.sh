#!/bin/bash
# Round 3 call: the pruned-kernel tests (incl. the async/capture test), the matrix A/B (new
# single-candidate top-k at 8 waves/SIMD vs the same at 4 vs the slot-based kernel), the
# config 5-T600 profile, then the deferral tuning A/B (tools/gpu_r3c.sh).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_ruby_mirror.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_b.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/t_b.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_matrix_ab.sh 2 base post_occ4 post_old || exit 2
bash tools/profile_round.sh r3b_config5_T600 --config 5-T600 || exit 3
echo r3b_done
bash tools/gpu_r3c.sh || exit 4
