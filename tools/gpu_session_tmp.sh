export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_corpus_sizes.py tests/test_gpu_slowpath.py -k "post or slow" -x -q --timeout 300 -m gpu > gpurun_out/t_pf.log 2>&1; echo pf_tests=$?; tail -2 gpurun_out/t_pf.log
bash tools/gpu_ab.sh 2 "--config 5-T600 --steps 10" base lib:nopf lib:m16o8
