// Decoded-path variant of the chain kernel, its traceback, and the chain launchers.
#include "chain_impl.h"

namespace svh {
namespace {

// Decoded-path variant: E in VGPRs, HA 1 (a model with no heavy feeder runs it too); P = 2 when
// every heavy term wins its ties (one compare per mask bit), 1 otherwise.
template <int W, int P>
const void* chain_paths_ptr_w(int sm) {
    switch (sm) {
#define SVH_CASE(SMV) \
    case SMV: return reinterpret_cast<const void*>(&chain_viterbi_kernel<SMV, W, 1, false, false, 0, P>);
        SVH_CASE(1) SVH_CASE(2) SVH_CASE(3) SVH_CASE(4) SVH_CASE(5)
#undef SVH_CASE
        default: return nullptr;
    }
}
template <int P>
const void* chain_paths_ptr(int sm, int waves) {
    switch (waves) {
        case 1: return chain_paths_ptr_w<1, P>(sm);
        case 2: return chain_paths_ptr_w<2, P>(sm);
        case 4: return chain_paths_ptr_w<4, P>(sm);
        case 8: return chain_paths_ptr_w<8, P>(sm);
        default: return nullptr;
    }
}
}  // namespace

const void* chain_paths_fn(int sm, int waves, bool ties_heavy) {
    return ties_heavy ? chain_paths_ptr<2>(sm, waves) : chain_paths_ptr<1>(sm, waves);
}


namespace {

constexpr uint32_t kTbMaxCap = 5 * 512;  // SM * B of the largest decoded-path geometry

// j*_h of record row r: the lowest light position p with fl(cA_h + v_r[p]) == fl(cA_h + mu_r),
// cA_h the light-set constant of heavy row h for the symbol of observation r+1 (the heavy row's
// light-set argmin, lexicographic (value, row) as the oracle).  v_r is recomputed by the wave
// from the checkpoint row c = r rounded down to kCkptEvery with the chain kernel's float
// operations: light v_i[p] = fminf(fl(fl(E + bw) + v_{i-1}[p-1]), fl(fl(E + aw) + vh_{i-1}[0])),
// heavy vh_i[h] = fminf(fl(cA + mu_{i-1}), fl(cX_h0 + vh_{i-1}[0]), fl(cX_h1 + vh_{i-1}[1])),
// mu = min of the light scores; vh_c comes from record row c.  buf: 2 * SM * B floats of LDS.
__device__ uint32_t recompute_jstar(const BandModel& m, const FusedBatch& b, uint32_t q, uint32_t r, uint32_t h,
                                   float* buf) {
    const uint32_t lane = threadIdx.x, SM = m.SM, B = m.B, cap = SM * B;
    const uint32_t* rec = b.hrec + b.hrec_off[q];
    const uint8_t* sym = b.symbols + b.sym_off[q];
    const uint32_t c = r / kCkptEvery * kCkptEvery;
    const float* ck = b.ckpt + b.ckpt_off[q] + (size_t)(c / kCkptEvery) * cap;
    float* cur = buf;
    float* nxt = buf + kTbMaxCap;
    for (uint32_t x = lane; x < cap; x += 64) cur[x] = ck[x];
    float vh0 = __builtin_bit_cast(float, rec[(size_t)c * kRecWords]);
    float vh1 = __builtin_bit_cast(float, rec[(size_t)c * kRecWords + 1]);
    __syncthreads();
    for (uint32_t i = c + 1; i <= r; ++i) {
        const float* e = m.erows + (size_t)sym[i] * m.erow;
        float pm = kInf;
        for (uint32_t x = lane; x < cap; x += 64) {
            const uint32_t sl = x / B, t = x % B;
            const float pv = sl ? cur[x - B] : (t ? cur[(SM - 1) * B + t - 1] : kInf);
            const float xb = (e[x] + m.bw[x]) + pv;
            nxt[x] = fminf(xb, (e[x] + m.aw[x]) + vh0);
            pm = fminf(pm, cur[x]);
        }
        for (int off = 32; off >= 1; off >>= 1) pm = fminf(pm, __shfl_xor(pm, off));
        const float* tl = e + cap;  // heavy constants of sym[i]
        float n0 = tl[kBandTailA + 0] + pm;
        n0 = fminf(n0, tl[band_tail_x(0, 0)] + vh0);
        n0 = fminf(n0, tl[band_tail_x(0, 1)] + vh1);
        float n1 = tl[kBandTailA + 1] + pm;
        n1 = fminf(n1, tl[band_tail_x(1, 0)] + vh0);
        n1 = fminf(n1, tl[band_tail_x(1, 1)] + vh1);
        vh0 = n0;
        vh1 = n1;
        float* tmp = cur;
        cur = nxt;
        nxt = tmp;
        __syncthreads();
    }
    const float mu = __builtin_bit_cast(float, rec[(size_t)r * kRecWords + 2]);
    const float ca = m.erows[(size_t)sym[r + 1] * m.erow + cap + kBandTailA + h];
    const float tgt = ca + mu;
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t x = lane; x < cap; x += 64)
        if (ca + cur[x] == tgt) best = min(best, (x % B) * SM + x / B);  // natural position
    for (int off = 32; off >= 1; off >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, off));
    __syncthreads();  // buf is reused by the next call
    return best;
}

// Path traceback over the decoded-path variant's records, one wave per sequence.  The walk is
// speculative along runs: inside a run of chain steps (light position p at observation i came
// from p-1 at i-1) or of heavy self-loops, lane l reads the record of observation i-l in
// parallel, and the first lane whose record leaves the run ends the iteration; so a sequence
// costs about (len / 64 + number of runs) dependent rounds of loads instead of len.  A heavy
// row whose light-set term wins or ties stops the run; if that lane is the first to stop, the
// wave recomputes its j* (recompute_jstar) and settles it.
__global__ __launch_bounds__(64) void chain_traceback_kernel(BandModel m, FusedBatch b, const uint64_t* path_off,
                                                              int32_t* paths) {
    __shared__ float buf[2 * kTbMaxCap];
    const uint32_t q = blockIdx.x, lane = threadIdx.x;
    if (b.run_mask && !b.run_mask[q]) return;  // rows the pipelined kernel traced itself
    const uint32_t len = b.end[q];
    const uint32_t SM = m.SM, B = m.B;
    const uint32_t* msk = b.cmask + b.cmask_off[q];
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
        bool cont = false, needj = false;
        float hv = kInf, lv = kInf;
        uint32_t hcol = 0xFFFFFFFFu;
        bool hex = false;
        if (pos >= 0) {  // light run: lane l looks at position pos-l at observation i-l
            const int64_t p = (int64_t)pos - (int64_t)lane;
            if (valid && p >= 0) {
                const uint32_t tt = (uint32_t)p / SM, ss = (uint32_t)p % SM;
                const uint32_t word = msk[(((uint64_t)r >> 5) * SM + ss) * B + tt];
                const uint32_t f = m.pflags[ss * B + tt];
                if ((word >> (31u - ((uint32_t)r & 31u))) & 1u) {
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
            // heavy-row terms fl(cX + vo[k]) and the light-set term fl(cA + mu).
            const uint32_t h = (uint32_t)(-1 - pos);
            const uint32_t* rw = rec + (uint64_t)r * kRecWords;
            const float vo[2] = {__builtin_bit_cast(float, rw[0]), __builtin_bit_cast(float, rw[1])};
            const float mu = __builtin_bit_cast(float, rw[2]);
            const float* tl = m.erows + (size_t)sym[r + 1] * m.erow + (size_t)SM * B;  // heavy constants
#pragma unroll
            for (int k = 0; k < kBandHeavy; ++k) {
                if ((m.hx_exist >> (h * kBandHeavy + k)) & 1u) {
                    const float val = tl[band_tail_x(h, k)] + vo[k];
                    const uint32_t col = (uint32_t)m.hrow[k];
                    const bool take = !hex || val < hv || (val == hv && col < hcol);
                    hv = take ? val : hv;
                    hcol = take ? col : hcol;
                    hex = true;
                }
            }
            pred = hex ? (int32_t)hcol : -1;
            if ((m.hl_exist >> h) & 1u) {
                lv = tl[kBandTailA + h] + mu;
                needj = !hex || !(hv < lv);  // the light set wins or ties: its lowest row j* decides
            }
            cont = !needj && pred == s;
        }
        uint64_t stop = __builtin_amdgcn_ballot_w64(!cont);
        uint32_t ls = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;  // first lane leaving the run
        while (ls < 64u && __builtin_amdgcn_readlane((int)needj, (int)ls)) {
            const uint32_t rs = (uint32_t)(i - 1 - (int64_t)ls);
            const uint32_t jp = recompute_jstar(m, b, q, rs, (uint32_t)(-1 - pos), buf);
            if (lane == ls) {
                const uint32_t js = m.lrow[(jp % SM) * B + jp / SM];
                const uint32_t k = !hex || lv < hv ? js : min(hcol, js);
                pred = k == 0xFFFFFFFFu ? -1 : (int32_t)k;
                cont = pred == s;
                needj = false;
            }
            stop = __builtin_amdgcn_ballot_w64(!cont);
            ls = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
        }
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
bool chain_paths_supported(int sm, int waves) { return chain_paths_fn(sm, waves, false) != nullptr; }

hipError_t launch_chain_traceback(const BandModel& m, const FusedBatch& b, const uint64_t* path_off,
                                  int32_t* paths, hipStream_t stream) {
    if (!b.cmask || !b.hrec || !b.ckpt || m.B % 64 || m.SM * m.B > kTbMaxCap || !m.spos || !m.pflags)
        return hipErrorInvalidValue;
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
        if (ge || ha != 1 || !b.hrec || !b.ckpt || !m.pflags) return hipErrorInvalidValue;
        fn = chain_paths_fn(sm, waves, m.ties_heavy != 0);
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
    // decoded paths stage their masks and heavy records in LDS
    const size_t lds = chain_lds_bytes() + (b.cmask ? chain_path_lds_bytes() : 0);
    return hipLaunchKernel(fn, dim3(b.nseq), dim3(m.B), args, lds, stream);
}

}  // namespace svh
