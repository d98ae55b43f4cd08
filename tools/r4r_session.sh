# round-4 session r: profiles of config 3 on the postings kernels (all pairs) and of 5-T600
DICE_POST_PRUNE=0 bash tools/profile_round.sh r4r_config3_post --config 3 && bash tools/profile_round.sh r4r_config5_T600 --config 5-T600
