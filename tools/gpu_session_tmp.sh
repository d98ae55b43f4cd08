export TMPDIR=/tmp
mkdir -p gpurun_out
LICENSEE_DICE_LIB=licensee_amd/lib/var/split12.so timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py -x -q --timeout 300 -m gpu -k "post" > gpurun_out/t_split.log 2>&1 || { echo tests failed; tail -20 gpurun_out/t_split.log; exit 3; }
tail -1 gpurun_out/t_split.log
bash tools/gpu_ab.sh 3 "--config 3 --steps 10" DICE_POST_PRUNE=0 lib:split12,DICE_POST_PRUNE=0
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base lib:split12
