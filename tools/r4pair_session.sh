# round-4 session: matrix scoring with two consecutive templates per lane (POST_PAIR_SCORE):
# parity of the T > 64 matrix paths, A/B against one template per lane (lib:nopair), trace
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_configs.py tests/test_gpu_slowpath.py tests/test_gpu_parity.py tests/test_gpu_upload_ids.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4pair_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4pair_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 3 "--config 5-T600 --steps 10" base lib:nopair || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4pair_5T600/trace -o run --output-format csv -- python bench.py --config 5-T600 --steps 10 --warmup 2 --no-cpu-baseline --no-extras --extra-configs= > gpurun_out/r4pair_trace.json 2> gpurun_out/r4pair_trace.err || exit 5
echo session_done
