export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_slowpath.py tests/test_gpu_confidence.py -x -q --timeout 300 -m gpu > gpurun_out/t_d20.log 2>&1; echo d20_tests=$?; tail -3 gpurun_out/t_d20.log
bash tools/gpu_ab.sh 2 "--config 3 --steps 10" DICE_POST_PRUNE=0,DICE_POST_DENSE=16 DICE_POST_PRUNE=0
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" DICE_POST_DENSE=16 base
