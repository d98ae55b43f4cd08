// Template-specialized sparse scoring program (declarations). See dice_program.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/licensee_dice.h"

namespace dice {

// One program entry: accumulate popcount(file_dword[dword] & mask) into template `tpl`.
struct Entry {
    int32_t tpl;
    int32_t dword;
    uint32_t mask;
};

struct Program {
    std::vector<Entry> prog;          // sorted by (dword, tpl)
    std::vector<int32_t> dword_map;   // vocab dword -> file dword in the remapped layout (-1: unused)
    int32_t wpb = 4;                  // waves (64-file tiles) per workgroup
    std::vector<int32_t> qperm;       // tile slot -> vocabulary quad (empty: identity)
    size_t entries() const { return prog.size(); }
};

int program_setup(dice_ctx* c, const dice_templates* t);
int program_launch_match(dice_ctx* c, dice_batch* b, double thr, hipStream_t s);
int program_launch_matrix(dice_ctx* c, dice_batch* b, int32_t k, hipStream_t s);

}  // namespace dice
