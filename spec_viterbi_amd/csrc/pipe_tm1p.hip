// Pipelined chain Viterbi kernel, pair tables (pipe_kernel.h TM = 4, the default; TM = 1 in
// SVH_PIPE_AB_ALL builds):
// decoded-path instantiations (PATHS 1 and 2), 2 slots per lane, 4 waves per workgroup.
// The LDS boundary ring of these instantiations is batched per group of 8 (SVH_PIPE_RING8 = 1: two
// ds_write_b128 per group instead of a ds_write_b32 per step).  With the pair-table step the
// per-step LDS store paced the pipeline: 0.363 -> 0.282 ms on the headline (profiles/r04_s4/ab.log;
// TM = 0 in pipe.hip keeps the per-step row, 0.335 vs 0.342 ms batched).
#ifndef SVH_PIPE_RING8
#define SVH_PIPE_RING8 1
#endif
#include "pipe_kernel.h"

namespace svh {

const void* pipe_kernel_tm1_paths(int sm, int waves, bool sx, int paths, int tm) {
#ifdef SVH_PIPE_AB_ONLY
    return nullptr;
#else
    if (sm != 2 || waves != 4 || paths < 1 || paths > 2) return nullptr;
    if (tm == 4) {  // indexed operands, packed feeder terms
        if (paths == 2)
            return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 2, 4>)
                      : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 2, 4>);
        return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 1, 4>)
                  : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 1, 4>);
    }
#ifdef SVH_PIPE_AB_ALL  // TM = 1 decoded paths (A/B: DESIGN.md 5f, 0.439 vs 0.412 ms for TM 4)
    if (paths == 2)
        return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 2, 1>)
                  : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 2, 1>);
    return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 1, 1>)
              : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 1, 1>);
#else
    return nullptr;
#endif
#endif
}

}  // namespace svh
