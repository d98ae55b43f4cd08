# round-4 session q: profiles (kernel trace + FETCH/WRITE/SQ/clock passes) of config 3 through
# both match entry points
bash tools/profile_round.sh r4q_config3 --config 3 && bash tools/profile_round.sh r4q_config3_top1 --config 3 --match-mode top1
