# round-4 session j: the dense prefix on the matrix cores (dice_post_dense_mfma, DICE_POST_MFMA)
# and the sparse program's tile queue (DICE_PROG_QUEUE): parity, then interleaved A/Bs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_configs.py tests/test_gpu_corpus_sizes.py tests/test_gpu_slowpath.py tests/test_gpu_confidence.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4j_tests.log; [ $rc -eq 0 ] || exit $rc
DICE_PROG_QUEUE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_golden.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4j_queue_tests.log 2>&1
rc=$?; echo "queue_tests_rc=$rc"; tail -2 gpurun_out/r4j_queue_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 2 "--config 3 --steps 20 --match-mode top1" DICE_POST_PRUNE=0 DICE_POST_PRUNE=0,DICE_POST_MFMA=0 base DICE_POST_MFMA=0 || exit 3
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base DICE_POST_MFMA=0 || exit 4
bash tools/gpu_ab.sh 3 "--config 2 --steps 50" base DICE_PROG_QUEUE=1 DICE_PROG_QUEUE=1,DICE_PROG_WPB=2 DICE_PROG_QUEUE=1,DICE_PROG_WPB=1 || exit 5
echo session_done
