# round-4 session d: matrix-mode parity (global row stores, top-2 per lane), then A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_slowpath.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4d_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" lib:orig lib:prev base lib:u2 lib:notop2 || exit 3
