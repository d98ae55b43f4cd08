# round-4 session h: dense prefixes staged through LDS + u8 partials with u16 overflow rows:
# parity, then A/B of each change (lib:phead = before both)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_golden.py tests/test_gpu_configs.py tests/test_gpu_prune.py tests/test_gpu_slowpath.py tests/test_gpu_upload_ids.py tests/test_gpu_sharded.py tests/test_gpu_confidence.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4h_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4h_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 2 "--config 3 --steps 20" lib:phead,DICE_POST_PRUNE=0 lib:noLdsP,DICE_POST_PRUNE=0 lib:noU8,DICE_POST_PRUNE=0 DICE_POST_PRUNE=0 lib:phead base || exit 3
bash tools/gpu_ab.sh 2 "--config 3 --steps 20 --confidence" base || exit 5
timeout -k 10 300 python -u tools/exp/prune_long_files.py 250000 > gpurun_out/r4h_long.txt 2>&1 || exit 6
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" lib:phead lib:noLdsP lib:noU8 base lib:nostore || exit 4
