// Chain kernel instantiations with one heavy feeder (every reference .chmm), plus the
// diagnostic builds (segment stamps, exchange ablations).
#include "chain_impl.h"

namespace svh {
namespace {
template <int HA>
const void* chain_ptr(int sm, int waves, bool ge) {
    switch (waves) {
        case 1: return chain_ptr_w<1, HA>(sm, ge);
        case 2: return chain_ptr_w<2, HA>(sm, ge);
        case 4: return chain_ptr_w<4, HA>(sm, ge);
        case 8: return chain_ptr_w<8, HA>(sm, ge);
        default: return nullptr;
    }
}
}  // namespace

const void* chain_fn_ha1(int sm, int waves, bool ge) { return chain_ptr<1>(sm, waves, ge); }

const void* chain_diag_fn(int sm, int waves, bool ge, uint32_t dbg) {
    const void* fn = nullptr;
    if (dbg & 4u) {  // diagnostic stamp builds
        if (!ge && sm == 5 && waves == 8) fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<5, 8, 1, false, true>);
        if (!ge && sm == 5 && waves == 1) fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<5, 1, 1, false, true>);
        if (ge && sm == 10 && waves == 4) fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<10, 4, 1, true, true>);
    }
    if ((dbg & (64u | 2048u | 4096u)) && !ge && sm == 5 && waves == 8) {  // diagnostic ablations
        switch (((dbg >> 6) & 1u) | ((dbg >> 10) & 6u)) {
            case 1: fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<5, 8, 1, false, false, 1>); break;
            case 2: fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<5, 8, 1, false, false, 2>); break;
            case 4: fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<5, 8, 1, false, false, 4>); break;
            case 6: fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<5, 8, 1, false, false, 6>); break;
            default: break;
        }
    }
    return fn;
}

}  // namespace svh
