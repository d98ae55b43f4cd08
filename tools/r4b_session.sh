# round-4 session e: DPP wave argmax parity + A/B; config-3 pruned-kernel phase clocks
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_slowpath.py tests/test_gpu_configs.py tests/test_gpu_prune.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/r4e_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" lib:prev lib:nodpp base || exit 3
bash tools/gpu_ab.sh 2 "--config 3 --steps 20" lib:nodpp,DICE_POST_PRUNE=0 DICE_POST_PRUNE=0 lib:nodpp base || exit 4
LICENSEE_DICE_LIB=licensee_amd/lib/var/pdiag8.so timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --extra-configs= --no-cpu-baseline --no-extras > gpurun_out/r4e_pdiag.json 2> gpurun_out/r4e_pdiag.err || exit 5
grep "prune4 phases" gpurun_out/r4e_pdiag.err | tail -2
