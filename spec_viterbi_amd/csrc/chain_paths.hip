// Decoded-path variant of the chain kernel, its traceback, and the chain launchers.
#include "chain_impl.h"

namespace svh {
namespace {

// Decoded-path variant: E in VGPRs, HA 1 (a model with no heavy feeder runs it too).
template <int W>
const void* chain_paths_ptr_w(int sm) {
    switch (sm) {
#define SVH_CASE(SMV) \
    case SMV: return reinterpret_cast<const void*>(&chain_viterbi_kernel<SMV, W, 1, false, false, 0, true>);
        SVH_CASE(1) SVH_CASE(2) SVH_CASE(3) SVH_CASE(4) SVH_CASE(5)
#undef SVH_CASE
        default: return nullptr;
    }
}
}  // namespace

const void* chain_paths_fn(int sm, int waves) {
    switch (waves) {
        case 1: return chain_paths_ptr_w<1>(sm);
        case 2: return chain_paths_ptr_w<2>(sm);
        case 4: return chain_paths_ptr_w<4>(sm);
        case 8: return chain_paths_ptr_w<8>(sm);
        default: return nullptr;
    }
}


namespace {

// Path traceback over the decoded-path variant's records, one wave per sequence.  The walk is
// speculative along runs: inside a run of chain steps (light position p at observation i came
// from p-1 at i-1) or of heavy self-loops, lane l reads the record of observation i-l in
// parallel, and the first lane whose record leaves the run ends the iteration; so a sequence
// costs about (len / 64 + number of runs) dependent rounds of loads instead of len.
__global__ __launch_bounds__(64) void chain_traceback_kernel(BandModel m, FusedBatch b, const uint64_t* path_off,
                                                              int32_t* paths) {
    const uint32_t q = blockIdx.x, lane = threadIdx.x;
    const uint32_t len = b.end[q];
    const uint32_t SM = m.SM, B = m.B, W = B / 64;
    const uint64_t* msk = b.cmask + b.cmask_off[q];
    const uint32_t* rec = b.hrec + b.hrec_off[q];
    int32_t* out = paths + path_off[q];
    const uint8_t* sym = b.symbols + b.sym_off[q];
    const int64_t best = b.best[q];
    int32_t s = best < 0 ? -1 : (int32_t)best;
    if (lane == 0) out[len - 1] = s;
    int64_t i = (int64_t)len - 1;  // out[i] == s is known; find out[i-1], out[i-2], ...
    while (i >= 1) {
        if (s < 0) {  // no predecessor: every earlier entry is -1 (oracle: ora_traceback)
            for (int64_t r = lane; r < i; r += 64) out[r] = -1;
            break;
        }
        const int32_t pos = m.spos[s];
        const int64_t r = i - 1 - (int64_t)lane;  // record row of this lane (observation r+1)
        const bool valid = r >= 0;
        int32_t pred = -1;
        bool cont = false;
        if (pos >= 0) {  // light run: lane l looks at position pos-l at observation i-l
            const int64_t p = (int64_t)pos - (int64_t)lane;
            if (valid && p >= 0) {
                const uint32_t tt = (uint32_t)p / SM, ss = (uint32_t)p % SM;
                const uint64_t word =
                    msk[((((uint64_t)r >> 5) * W + tt / 64) * 32 + ((uint32_t)r & 31u)) * SM + ss];
                const uint32_t f = m.pflags[ss * B + tt];
                if ((word >> (tt & 63u)) & 1ull) {
                    pred = m.hrow[0];
                } else if ((f & 1u) && p >= 1) {
                    const uint32_t pp = (uint32_t)p - 1;
                    pred = (int32_t)m.lrow[(pp % SM) * B + pp / SM];
                    cont = true;
                }
            }
        } else if (valid) {  // heavy run: self-loops of heavy row h
            // The heavy row's lexicographic (value, row) argmin at observation r+1, re-evaluated
            // from the recorded inputs with the kernel's float operations (heavy_update): the
            // heavy-row terms fl(cX + vo[k]) and the light-set term fl(cA + mu), whose lowest row
            // is the recorded j* (a light position).
            const uint32_t h = (uint32_t)(-1 - pos);
            const uint32_t* rw = rec + (uint64_t)r * kRecWords;
            const float vo[2] = {__builtin_bit_cast(float, rw[0]), __builtin_bit_cast(float, rw[1])};
            const float mu = __builtin_bit_cast(float, rw[2]);
            const uint32_t o = sym[r + 1];
            const float* tl = m.erows + (size_t)o * m.erow + (size_t)SM * B;  // heavy constants of o
            float hv = kInf;
            uint32_t hcol = 0xFFFFFFFFu;
            bool hex = false;
#pragma unroll
            for (int k = 0; k < kBandHeavy; ++k) {
                if ((m.hx_exist >> (h * kBandHeavy + k)) & 1u) {
                    const float val = tl[kBandTailX + h * kBandHeavy + k] + vo[k];
                    const uint32_t col = (uint32_t)m.hrow[k];
                    const bool take = !hex || val < hv || (val == hv && col < hcol);
                    hv = take ? val : hv;
                    hcol = take ? col : hcol;
                    hex = true;
                }
            }
            uint32_t k = hex ? hcol : 0xFFFFFFFFu;
            if ((m.hl_exist >> h) & 1u) {
                const float lv = tl[kBandTailA + h] + mu;
                if (!hex || !(hv < lv)) {  // the light set wins or ties: its lowest row j*
                    const uint32_t jp = rw[kRecJ + h];
                    const uint32_t js = m.lrow[(jp % SM) * B + jp / SM];
                    k = !hex || lv < hv ? js : min(hcol, js);
                }
            }
            pred = k == 0xFFFFFFFFu ? -1 : (int32_t)k;
            cont = pred == s;
        }
        const uint64_t stop = __builtin_amdgcn_ballot_w64(!cont);
        const uint32_t ls = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;  // first lane leaving the run
        // entries written this round: the run's lanes plus the leaving lane if it has a record
        const uint32_t k = ls == 64u ? 64u : ((int64_t)ls <= i - 1 ? ls + 1u : ls);
        if (lane < k) out[r] = pred;
        s = __builtin_amdgcn_readlane(pred, (int)(k - 1u));
        i -= (int64_t)k;
    }
}

}  // namespace

bool chain_supported(int sm, int waves, int ha, bool ge) {
    return (ha == 1 ? chain_fn_ha1(sm, waves, ge) : ha == 2 ? chain_fn_ha2(sm, waves, ge) : nullptr) != nullptr;
}
bool chain_paths_supported(int sm, int waves) { return chain_paths_fn(sm, waves) != nullptr; }

hipError_t launch_chain_traceback(const BandModel& m, const FusedBatch& b, const uint64_t* path_off,
                                  int32_t* paths, hipStream_t stream) {
    if (!b.cmask || !b.hrec || m.B % 64 || !m.spos || !m.pflags) return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    hipLaunchKernelGGL(chain_traceback_kernel, dim3(b.nseq), dim3(64), 0, stream, m, b, path_off, paths);
    return hipGetLastError();
}

hipError_t launch_chain(const BandModel& m, int ha, const FusedBatch& b, hipStream_t stream) {
    const int waves = (int)(m.B / 64);
    const bool ge = m.ge != 0;
    const int sm = (int)m.SM;
    const void* fn = ha == 1 ? chain_fn_ha1(sm, waves, ge) : ha == 2 ? chain_fn_ha2(sm, waves, ge) : nullptr;
    if (b.cmask) {  // decoded paths
        if (ge || ha != 1 || !b.hrec || !m.pflags) return hipErrorInvalidValue;
        fn = chain_paths_fn(sm, waves);
    } else if (ha == 1 && (m.dbg & (4u | 64u | 2048u | 4096u))) {
        if (const void* d = chain_diag_fn(sm, waves, ge, m.dbg)) fn = d;
    }
    if (!fn || m.B % 64 || m.S > (uint32_t)kChainMaxSym || m.erow < m.SM * m.B + kBandTail ||
        (ge && !m.erows_t))
        return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    BandModel mm = m;
    FusedBatch bb = b;
    void* args[] = {&mm, &bb};
    // decoded paths keep the light scores of two observations in LDS
    const size_t lds = chain_lds_bytes() + (b.cmask ? chain_path_lds_bytes(m.B / 64, m.SM) : 0);
    return hipLaunchKernel(fn, dim3(b.nseq), dim3(m.B), args, lds, stream);
}

}  // namespace svh
