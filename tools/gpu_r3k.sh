#!/bin/bash
# Round 3 final measurement set on the final code: the default bench line with a same-lease trace and
# the config-2 profile (tools/gpu_measure.sh r3k "2"), then the config-3 all-pairs profile (postings
# kernels, DICE_POST_PRUNE=0) for pmc_config3_post.json.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_measure.sh r3k "2" || exit $?
DICE_POST_PRUNE=0 bash tools/profile_round.sh r3k_config3_post --config 3 || exit 9
echo r3k_done
