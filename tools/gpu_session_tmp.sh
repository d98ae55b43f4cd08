export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py -k "post" -x -q --timeout 300 -m gpu > gpurun_out/t_ahead.log 2>&1; echo ahead_tests=$?; tail -2 gpurun_out/t_ahead.log
LICENSEE_DICE_LIB=licensee_amd/lib/var/ahead1c4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py -k "post and 700" -x -q --timeout 300 -m gpu > gpurun_out/t_ahead4.log 2>&1; echo ahead4_tests=$?; tail -2 gpurun_out/t_ahead4.log
bash tools/gpu_ab.sh 2 "--config 3 --steps 10" DICE_POST_PRUNE=0 lib:ahead0,DICE_POST_PRUNE=0 lib:ahead1c4,DICE_POST_PRUNE=0
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base lib:ahead0
