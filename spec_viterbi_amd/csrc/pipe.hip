// Pipelined chain Viterbi kernel (gfx950), TM = 0 instantiations and the launch: the kernel
// template and its documentation are in pipe_kernel.h; pipe_tm1.hip / pipe_tm1p.hip instantiate
// the pair-table variant (TM = 1).
#include "pipe_kernel.h"

#include <cstdlib>

namespace svh {

namespace {

template <int SM, int W, int PATHS = 0>
const void* pipe_ptr(bool sx) {
    return sx ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<SM, W, true, PATHS, 0>)
              : reinterpret_cast<const void*>(&pipe_viterbi_kernel<SM, W, false, PATHS, 0>);
}

}  // namespace

// paths: 0 scores only, 1 decoded paths, 2 decoded paths where F wins every tie
const void* pipe_kernel_tm0(int sm, int waves, bool sx, int paths) {
#ifdef SVH_PIPE_AB_ONLY  // A/B timing builds: the headline geometry only (compile time)
    return sm == 2 && waves == 4 && !sx && !paths ? reinterpret_cast<const void*>(&pipe_viterbi_kernel<2, 4, false, 0, 0>)
                                                  : nullptr;
#else
    if (paths) {  // decoded-path variant: the default geometry only (2 slots, 4 waves)
        if (sm != 2 || waves != 4) return nullptr;
        return paths == 2 ? pipe_ptr<2, 4, 2>(sx) : pipe_ptr<2, 4, 1>(sx);
    }
    switch (sm * 100 + waves) {
        case 204: return pipe_ptr<2, 4>(sx);  // the geometry AUTO plans (alphabets of 21..32 symbols)
#ifdef SVH_PIPE_AB_ALL  // A/B and geometry-test builds: the geometries measured against it
        case 104: return pipe_ptr<1, 4>(sx);
        case 108: return pipe_ptr<1, 8>(sx);
        case 208: return pipe_ptr<2, 8>(sx);
#endif
        default: return nullptr;
    }
#endif
}

bool pipe_supported(int sm, int waves, bool sx) { return pipe_kernel_tm0(sm, waves, sx, 0) != nullptr; }
bool pipe_tm_supported(int tm) {
    if (tm == 0) return true;
    if (tm == -8) return pipe_kernel_tm1(2, 8, false, -4) != nullptr;  // TM 4 at 8 waves (A/B builds)
    return tm >= 1 && tm <= 4 && pipe_kernel_tm1(2, 4, false, tm >= 2 ? -tm : 0) != nullptr;
}
bool pipe_paths_supported(int sm, int waves) { return pipe_kernel_tm0(sm, waves, false, 1) != nullptr; }

hipError_t launch_pipe(const PipeModel& m, const FusedBatch& b, const PipeScratch& x, hipStream_t stream,
                       bool step_floor) {
    const bool paths = b.cmask != nullptr;
    const int pv = paths ? (m.ties_heavy ? 2 : 1) : 0;
    // TM = 1 (pair tables) needs 2 slots per lane and at most kPairSym symbols
    if (m.tm && (m.SM != 2 || m.S > kPairSym)) return hipErrorInvalidValue;
    if (step_floor && (paths || m.tm != 4 || m.W != 4)) return hipErrorInvalidValue;
    const void* fn = step_floor ? pipe_kernel_floor(m.sx != 0)
                     : !m.tm ? pipe_kernel_tm0((int)m.SM, (int)m.W, m.sx != 0, pv)
                     : paths ? pipe_kernel_tm1_paths((int)m.SM, (int)m.W, m.sx != 0, pv, m.tm == 4 ? 4 : 1)
                             : pipe_kernel_tm1((int)m.SM, (int)m.W, m.sx != 0, m.tm >= 2 ? -(int)m.tm : 0);
    if (!fn || m.S > 32 || m.G == 0 || m.nblk > m.G * m.W || m.P != m.nblk * 64 * m.SM || !x.ctr ||
        b.nseq > x.rows || x.G < m.G)
        return hipErrorInvalidValue;
    if (paths && (!b.ckpt || !b.prec || !b.fck || !m.pflags)) return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    PipeModel mm = m;
    FusedBatch bb = b;
    PipeScratch xx = x;
    void* args[] = {&mm, &bb, &xx};
    uint64_t grid = (uint64_t)b.nseq * m.G;
    // XCD-class mapping of rows to workgroups when the launch fits the chip at one workgroup per CU
    // (pipe_kernel.h: per-class tickets in start order, deadlock-free whatever else holds CUs; the
    // size condition is about speed only); SVH_PIPE_XMAP=0 keeps the single ticket counter (A/B)
    static const bool xmap_env = !(std::getenv("SVH_PIPE_XMAP") && std::atoi(std::getenv("SVH_PIPE_XMAP")) == 0);
    // (the grid padded to a multiple of 8, equal classes: pipe_kernel.h; padding slots exit at once)
    const uint64_t padded = (grid + 7) & ~7ull;
    xx.xmap = xmap_env && m.cus && padded <= m.cus ? 1u : 0u;
    if (xx.xmap) grid = padded;
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const size_t lds = paths ? (pipe_lds_bytes(m.W, m.S) + 15) / 16 * 16 + pipe_path_lds_bytes(m.W)
                             : pipe_lds_bytes(m.W, m.S);
    if (lds > 64 * 1024) {  // more than 64 KiB of dynamic LDS: a host-side attribute of the function
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    return hipLaunchKernel(fn, dim3((uint32_t)grid), dim3(64 * m.W), args, lds, stream);
}

}  // namespace svh
