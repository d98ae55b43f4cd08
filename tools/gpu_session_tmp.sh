export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab.sh 2 "--config 3 --steps 10" DICE_POST_PRUNE=0 lib:qu1,DICE_POST_PRUNE=0 lib:qu4,DICE_POST_PRUNE=0 DICE_POST_PRUNE=0,DICE_POST_MFMA_MT=2
