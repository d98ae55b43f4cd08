# round-4 session ab: MFMA dense prefix with 3 M-tiles per tile (DICE_POST_MFMA_MT=3): parity, A/B, trace
export TMPDIR=/tmp
mkdir -p gpurun_out
DICE_POST_MFMA_MT=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_corpus_sizes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4ab_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4ab_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 2 "--config 3 --steps 20 --match-mode top1" DICE_POST_PRUNE=0 DICE_POST_PRUNE=0,DICE_POST_MFMA_MT=3 || exit 3
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base DICE_POST_MFMA_MT=3 || exit 4
DICE_POST_MFMA_MT=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4ab_5T600/trace -o run --output-format csv -- python bench.py --config 5-T600 --steps 10 --warmup 2 --no-cpu-baseline --no-extras --extra-configs= > gpurun_out/r4ab_trace.json 2> gpurun_out/r4ab_trace.err || exit 5
echo session_done
