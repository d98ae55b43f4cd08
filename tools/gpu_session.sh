# round-6 session: GPU suite + smoke + default bench line, then the fusion-cost probe A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err; echo "bench_rc=$?"
tail -c 400 gpurun_out/r6a_bench.json
DICE_POST_PRUNE=0 bash tools/gpu_ab.sh 2 "--config 3 --steps 20" base lib:fnone lib:fprobe || exit $?
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base lib:fnone lib:fprobe
