// Wide pipelined chain Viterbi kernel (gfx950): scores-only instantiations and the launcher.  The
// kernel template and its documentation are in pipe_wide_kernel.h; pipe_wide_paths.hip
// instantiates the decoded-path variants.
#include "pipe_wide_kernel.h"

#include <cstdlib>

namespace svh {

namespace {

const void* pipew_fn(int sm, int waves, bool sx) {
    switch (sm * 100 + waves) {
        case 816: return pipew_ptr<8, 16, 0>(sx);
        case 812: return pipew_ptr<8, 12, 0>(sx);
        case 808: return pipew_ptr<8, 8, 0>(sx);
        case 804: return pipew_ptr<8, 4, 0>(sx);
        case 802: return pipew_ptr<8, 2, 0>(sx);
        case 801: return pipew_ptr<8, 1, 0>(sx);
        default: return nullptr;
    }
}

}  // namespace

bool pipew_supported(int sm, int waves, bool sx) { return pipew_fn(sm, waves, sx) != nullptr; }

bool pipew_paths_supported(int sm, uint32_t S, bool sx) { return pipew_paths_waves_max(sm, S, sx) != 0; }

uint32_t pipew_paths_waves_max(uint32_t sm, uint32_t S, bool sx) {
    for (uint32_t w = 8; w >= 1; w >>= 1)
        if (pipew_kernel_paths((int)sm, (int)w, sx, 1) && pipew_kernel_paths((int)sm, (int)w, sx, 2) &&
            pipew_lds_bytes(sm, w, S, sx, true) <= 160 * 1024)
            return w;
    return 0;
}

// b.cmask != nullptr: the decoded-path variant (PATHS 2 when F wins every tie, m.ties_heavy), with
// at most pipew_paths_waves_max sequences per workgroup.
hipError_t launch_pipew(const PipeModel& m, const FusedBatch& b, const PipeScratch& x, hipStream_t stream) {
    const bool paths = b.cmask != nullptr;
    uint32_t W = pipew_waves_for(m, b.nseq);
    if (paths) {
        const uint32_t wmax = pipew_paths_waves_max(m.SM, m.S, m.sx != 0);
        if (!wmax || !b.ckpt || !b.prec || !b.fck || !m.pflags) return hipErrorInvalidValue;
        W = W < wmax ? W : wmax;
    }
    const void* fn = paths ? pipew_kernel_paths((int)m.SM, (int)W, m.sx != 0, m.ties_heavy ? 2 : 1)
                           : pipew_fn((int)m.SM, (int)W, m.sx != 0);
    const size_t lds = pipew_lds_bytes(m.SM, W, m.S, m.sx != 0, paths);
    if (!fn || m.S > 32 || m.nblk == 0 || m.G != m.nblk || m.P != m.nblk * 64 * m.SM || !x.ctr ||
        b.nseq > x.rows || x.G < m.nblk || lds > 160 * 1024)
        return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    // more than 64 KiB of dynamic LDS must be allowed for the function (a host-side attribute)
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    PipeModel mm = m;
    mm.W = W;
    FusedBatch bb = b;
    PipeScratch xx = x;
    const void* hc = m.hc;
    void* args[] = {&mm, &bb, &xx, &hc};
    uint64_t groups = ((uint64_t)b.nseq + W - 1) / W;
    // XCD classes (pipe_wide_kernel.h): groups padded to a multiple of 8, class r = b % 8 takes a
    // contiguous eighth of them; SVH_PIPEW_XMAP=0 keeps the single ticket counter (A/B)
    static const bool xmap_env = !(std::getenv("SVH_PIPEW_XMAP") && std::atoi(std::getenv("SVH_PIPEW_XMAP")) == 0);
    xx.xmap = xmap_env ? 1u : 0u;
    if (xx.xmap) groups = (groups + 7) & ~7ull;
    const uint64_t grid = groups * m.nblk;
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    return hipLaunchKernel(fn, dim3((uint32_t)grid), dim3(64 * W), args, lds, stream);
}

}  // namespace svh
