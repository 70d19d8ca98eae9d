// Pipelined chain Viterbi kernel, TM = 1 (pair tables read by 64-bit moves; pipe_kernel.h):
// scores-only instantiations, 2 slots per lane, 4 waves per workgroup (one per SIMD: the 258
// registers of the pair tables do not fit the 256 of two waves per SIMD, which spilled).
#include "pipe_kernel.h"

namespace svh {

const void* pipe_kernel_tm1(int sm, int waves, bool sx, int paths) {
    if (sm != 2 || (paths && paths != -2)) return nullptr;
#ifdef SVH_PIPE_AB_ONLY  // A/B timing builds: the headline geometry only
    if (paths == -2) return waves == 4 && !sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 2>) : nullptr;
    return waves == 4 && !sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 1>) : nullptr;
#else
    if (waves != 4) return nullptr;
    if (paths == -2)  // TM = 2 (indexed operands; A/B: SVH_PIPE_TM=2)
        return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 0, 2>)
                  : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 2>);
    return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 0, 1>)
              : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 1>);
#endif
}

}  // namespace svh
