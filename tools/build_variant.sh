#!/bin/bash
# Build liblicensee_dice.so with extra compile flags into licensee_amd/lib/var/<name>.so, for
# A/B runs of compile-time kernel variants on the GPU box (LICENSEE_DICE_LIB=<path>).
#   tools/build_variant.sh <name> [-DFLAG=...]...
set -e
# POST_SRC=<file> / PRUNE_SRC=<file> build with another dice_post.hip / dice_prune.hip (e.g. a
# previous revision from git show).
NAME=$1; shift
cd "$(dirname "$0")/.."
mkdir -p licensee_amd/lib/var
C=licensee_amd/csrc
POST=${POST_SRC:-$C/dice_post.hip}
PRUNE=${PRUNE_SRC:-$C/dice_prune.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -I$C "$@" -o licensee_amd/lib/var/$NAME.so \
  $C/dice.hip $C/dice_lds.hip $POST $PRUNE $C/dice_exact.hip $C/dice_words.hip $C/dice_program.cpp $C/dice_shard.cpp -lhiprtc
echo licensee_amd/lib/var/$NAME.so
