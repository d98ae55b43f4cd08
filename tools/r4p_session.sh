# round-4 session p: full GPU suite + smoke, then the measurement set (default bench line,
# same-lease trace of config 2, config 2 profile)
bash tools/gpu_tests.sh && bash tools/gpu_measure.sh r4p "2"
