export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab.sh 3 "--config 5-T600 --steps 10" base lib:ms7
