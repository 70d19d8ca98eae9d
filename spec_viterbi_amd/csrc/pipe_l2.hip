// _spec level 2 on the pipelined latency plan: pipe_kernel.h with L2 = true (the pair-table scores
// kernel, TM = 4 geometry, 2 slots x 4 waves per workgroup), one launch for every chunk of every
// row.  The chunk step, its exactness argument and its checks are in pipe_kernel.h (step2).
#ifndef SVH_PIPE_RING8
#define SVH_PIPE_RING8 1
#endif
#include "pipe_kernel.h"

namespace svh {

bool pipe_l2_supported(const PipeModel& m) {
    return !m.wide && m.SM == 2 && m.W == 4 && m.S <= kPairSym && m.emax2 < kInf && m.G > 0;
}

hipError_t launch_pipe_l2(const PipeModel& m, const FusedBatch& b, const PipeScratch& x, hipStream_t stream) {
    if (!pipe_l2_supported(m) || m.nblk > m.G * m.W || m.P != m.nblk * 64 * m.SM || !x.ctr || b.nseq > x.rows ||
        x.G < m.G || b.cmask)
        return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    const void* fn = m.sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, true, 0, 4, true>)
                          : reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 4, true>);
    PipeModel mm = m;
    FusedBatch bb = b;
    PipeScratch xx = x;
    void* args[] = {&mm, &bb, &xx};
    uint64_t grid = (uint64_t)b.nseq * m.G;
    // rows mapped by XCD class when the launch fits the chip at one workgroup per CU (launch_pipe)
    const uint64_t padded = (grid + 7) & ~7ull;
    xx.xmap = m.cus && padded <= m.cus ? 1u : 0u;
    if (xx.xmap) grid = padded;
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    return hipLaunchKernel(fn, dim3((uint32_t)grid), dim3(64 * m.W), args, pipe_lds_bytes(m.W, m.S), stream);
}

}  // namespace svh
