// Decoded-path instantiations of the wide pipelined kernel (pipe_wide_kernel.h, PATHS = 1: ties
// by the per-position rule, 2: F wins every tie).
#include "pipe_wide_kernel.h"

namespace svh {

const void* pipew_kernel_paths(int sm, int waves, bool sx, int paths) {
    if (sm != 8 || (paths != 1 && paths != 2)) return nullptr;
    switch (waves * 10 + paths) {
        case 81: return pipew_ptr<8, 8, 1>(sx);
        case 82: return pipew_ptr<8, 8, 2>(sx);
        case 41: return pipew_ptr<8, 4, 1>(sx);
        case 42: return pipew_ptr<8, 4, 2>(sx);
        case 21: return pipew_ptr<8, 2, 1>(sx);
        case 22: return pipew_ptr<8, 2, 2>(sx);
        case 11: return pipew_ptr<8, 1, 1>(sx);
        case 12: return pipew_ptr<8, 1, 2>(sx);
        default: return nullptr;
    }
}

}  // namespace svh
