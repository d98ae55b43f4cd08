# round-4 session y: MFMA dense prefix with the two-VALU-per-dword widening (widen_half): parity,
# A/B against the nibble-multiply widening (lib:wid16), trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_corpus_sizes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4y_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4y_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 2 "--config 3 --steps 20 --match-mode top1" DICE_POST_PRUNE=0 lib:wid16,DICE_POST_PRUNE=0 || exit 3
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base lib:wid16 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4y_5T600/trace -o run --output-format csv -- python bench.py --config 5-T600 --steps 10 --warmup 2 --no-cpu-baseline --no-extras --extra-configs= > gpurun_out/r4y_trace.json 2> gpurun_out/r4y_trace.err || exit 5
echo session_done
