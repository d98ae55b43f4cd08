# round-4 session i: the sparse program's tile queue (DICE_PROG_QUEUE=1): parity of every
# sparse-program corpus with the queue on, an interleaved config-2 A/B (workgroup sizes), then
# profiles of config 3 through both match entry points (confidence = default, top1)
export TMPDIR=/tmp
mkdir -p gpurun_out
DICE_PROG_QUEUE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_corpus_sizes.py tests/test_gpu_golden.py tests/test_gpu_api.py tests/test_gpu_confidence.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4i_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4i_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 3 "--config 2 --steps 50" base DICE_PROG_QUEUE=1 DICE_PROG_QUEUE=1,DICE_PROG_WPB=2 DICE_PROG_QUEUE=1,DICE_PROG_WPB=1 DICE_PROG_WPB=2 || exit 3
bash tools/profile_round.sh r4i_config3 --config 3 || exit 4
bash tools/profile_round.sh r4i_config3_top1 --config 3 --match-mode top1 || exit 5
