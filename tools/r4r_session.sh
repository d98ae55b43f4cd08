# round-4 session r: the final measurement set -- default bench line + same-lease trace of
# config 2 (gpu_measure.sh with no per-config profiles), then profiles of config 3 on the
# postings kernels (all pairs) and of 5-T600
bash tools/gpu_measure.sh r4r "" && DICE_POST_PRUNE=0 bash tools/profile_round.sh r4r_config3_post --config 3 && bash tools/profile_round.sh r4r_config5_T600 --config 5-T600
