# round-4 session c: T > 64 postings-kernel parity after the matrix-kernel register work, then A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_configs.py tests/test_gpu_prune.py tests/test_gpu_golden.py tests/test_gpu_slowpath.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4c_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" lib:orig base lib:u1 lib:u5 lib:u10 || exit 3
bash tools/gpu_ab.sh 2 "--config 3 --steps 20" lib:orig,DICE_POST_PRUNE=0 DICE_POST_PRUNE=0 lib:orig base || exit 4
