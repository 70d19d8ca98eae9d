// Pipelined chain Viterbi kernel, pair tables (pipe_kernel.h TM = 4, the default; TM = 1..3 in
// SVH_PIPE_AB_ALL builds only): scores-only instantiations, 2 slots per lane, 4 waves per workgroup
// (one per SIMD: the 258 registers of the pair tables do not fit the 256 of two waves per SIMD).
// The LDS boundary ring of these instantiations is batched per group of 8 (SVH_PIPE_RING8 = 1: two
// ds_write_b128 per group instead of a ds_write_b32 per step).  With the pair-table step the
// per-step LDS store paced the pipeline: 0.363 -> 0.282 ms on the headline (profiles/r04_s4/ab.log;
// TM = 0 in pipe.hip keeps the per-step row, 0.335 vs 0.342 ms batched).
#ifndef SVH_PIPE_RING8
#define SVH_PIPE_RING8 1
#endif
#include "pipe_kernel.h"

namespace svh {

// The step-floor variant of the default (TM = 4) scores kernel (pipe_kernel.h FLOOR).
const void* pipe_kernel_floor(bool sx) {
    return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 0, 4, false, true>)
              : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 4, false, true>);
}

const void* pipe_kernel_tm1(int sm, int waves, bool sx, int paths) {
    if (sm != 2 || (paths && (paths < -4 || paths > -2))) return nullptr;
#ifdef SVH_PIPE_AB_ONLY  // A/B timing builds: the headline geometry only
    if (paths == -2) return waves == 4 && !sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 2>) : nullptr;
    if (paths == -3) return waves == 4 && !sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 3>) : nullptr;
    if (paths == -4) return waves == 4 && !sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 4>) : nullptr;
    return waves == 4 && !sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 1>) : nullptr;
#else
#ifndef SVH_PIPE_AB_ALL
    if (waves != 4) return nullptr;
#endif
    if (paths == -4 && waves == 4)  // TM = 4 (indexed operands, packed feeder terms): the mode AUTO selects
        return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 0, 4>)
                  : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 4>);
#ifdef SVH_PIPE_AB_ALL  // A/B and table-mode-test builds: the modes measured against it
    if (paths == -4 && waves == 8)  // TM = 4 at 8 waves per workgroup (two per SIMD: 3 workgroups per row)
        return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 8, true, 0, 4>)
                  : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 8, false, 0, 4>);
    if (waves != 4) return nullptr;
    if (paths == -2)  // TM = 2 (indexed operands; SVH_PIPE_TM=2)
        return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 0, 2>)
                  : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 2>);
    if (paths == -3)  // TM = 3 (packed feeder terms; SVH_PIPE_TM=3)
        return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 0, 3>)
                  : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 3>);
    if (paths == 0)  // TM = 1 (pair tables by 64-bit moves; SVH_PIPE_TM=1)
        return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 0, 1>)
                  : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 1>);
#endif
    return nullptr;
#endif
}

}  // namespace svh
