#!/bin/bash
# Round 3: narrow match kernel with per-tile result stores (LDS-parked results) and single-base
# copy-in: postings parity tests, then A/B against the committed dice_post.hip (post_head.so) on
# config 3 all pairs (DICE_POST_PRUNE=0), the default pruned match (deferred pass) and 5-T600.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_prune.py tests/test_gpu_slowpath.py tests/test_gpu_upload_ids.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_i.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/t_i.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base post_head; do
    if [ "$v" = base ]; then unset LICENSEE_DICE_LIB; else export LICENSEE_DICE_LIB=licensee_amd/lib/var/$v.so; fi
    timeout -k 10 300 python -u tools/exp/prune_ab.py --reps 2 --profiles 0 pruned post:DICE_POST_PRUNE=0 2>&1 | grep " ms " | sed "s/^/$v rep$rep: /" || exit 4
  done
done
unset LICENSEE_DICE_LIB
bash tools/gpu_matrix_ab.sh 2 base post_head || exit 2
