# round-4 session f: pruned-kernel parity (records 128-255 prefetched, speculative slot keys), A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_configs.py tests/test_gpu_corpus_sizes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4f_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 3 "--config 3 --steps 20" lib:pprev lib:nospec base lib:spec2 lib:g70 lib:g95 || exit 3
