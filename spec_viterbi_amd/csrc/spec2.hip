// _spec level 2 without the dense products (gfx950): each chunk's (min,+) product is evaluated
// from the two folded sparse matrices on chip, one persistent workgroup per sequence.
//
// Reference: Viterbi_impl/GraphBLAS_spec_impl.cpp.
//   add_level (:15-36): H_{(s1,s2)} = M_{s2} (x) M_{s1}, i.e. H[j][m] = min_p fl(A[j][p] + B[p][m])
//     with A = M_{s2}, B = M_{s1}, M_s[j][p] = fl(E_s[j] + T^T[j][p]) (:146-161);
//   run_Viterbi_spec (:66-81): per chunk of two observations v'[j] = min_m fl(H[j][m] + v[m]).
// fl(x + v) is monotone in x, so fl(min_p X_p + v) = min_p fl(X_p + v) and, bit for bit,
//     v'[j] = min_{p in in(j)} min_{m in in(p)} fl( fl(A[j][p] + B[p][m]) + v[m] )        (1)
// with +inf where no term exists (a structurally absent H entry contributes nothing, an entry of
// +inf contributes +inf).  The product is never formed: per chunk the terms of (1) are the
// two-hop paths j <- p <- m of the transition graph.
//
// Heavy rows (in-degree > kSpec2LightMax; N and C of the MSV models, ~2,406 terms each) would make
// (1) cost |in(p)| per (j, p) pair, 5.8 M terms per chunk on 2405.chmm.  With every score >= 0
// (all of T^T, E and the start scores non-negative: the reference's -log2 p, checked on the host)
// the inner minimum g_p(a) = min_{m in in(p)} fl(fl(a + b_m) + v_m) only depends on the few m whose
// c_m = b_m + v_m is near the smallest: for a >= 0, b, v >= 0 each fl() is within (1 +- u) of the
// exact sum (u = 2^-24, no cancellation), so F_m = fl(fl(a + b_m) + v_m) lies in
// [T_m (1-u)^2, T_m (1+u)^2], T_m = a + c_m.  With c_f = fl(b + v) and
//     theta = c_f_min + max((amax_p + c_f_min) 2^-20, 2^-126),   amax_p >= every finite a of p,
// any m with c_f_m > theta has F_m > F_{m*} for m* = argmin c_f (the margin 16u(amax + c_f_min)
// exceeds the ~4u a + 7u c_f_min that the roundings can close), so dropping it changes no bit of
// g_p.  Per chunk and heavy row: one pass over its terms (c_f and their minimum), one compaction of
// the candidates (c_f <= theta; usually 1-3), and every (j, p) pair loops over p's candidates only.
// A model with any negative score runs with theta = +inf (every term a candidate): still (1),
// exactly, just without the pruning.
//
// Per chunk (symbols s1 = seq[1+2c], s2 = seq[2+2c]), three barriers:
//   1  light rows p: pairs LP[p][k] = (b, v_m) = (fl(E_s1[p] + T^T[p][m_k]), v[m_k]);
//      heavy terms x of row p: HP[x] = (b, v_m), c_f = fl(b + v_m), a per-row minimum (LDS atomic);
//   1b heavy terms: candidates c_f <= theta appended to CL[row's range] (wave-aggregated atomics);
//   2  light rows j: v'[j] = min over its terms p of the loop over LP[p] (light p) or CL[p] (heavy
//      p); heavy terms (j, p): the same per term, then a per-row minimum into hacc[j].
// Scores of heavy rows live in hacc (order-preserving keys, LDS ds_min_u32), light rows in vl.
#include "device_common.h"
#include "kernels.h"

namespace svh {

using namespace dev;

namespace {

constexpr uint32_t kS2Threads = kSpec2Threads;
constexpr uint32_t kNone = 0xFFFFFFFFu;

// order-preserving key of a float (unsigned order == float order, -0 below +0): ds_min_u32 on keys
// is a float minimum with no denormal or signed-zero ambiguity
__device__ __forceinline__ uint32_t okey(float f) {
    const uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float okey_val(uint32_t k) {
    return __builtin_bit_cast(float, (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ __forceinline__ void lds_min_u32(uint32_t* p, uint32_t v) {
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the candidate bound of a heavy row (see the header); cmin = +inf: no term can be finite
__device__ __forceinline__ float theta_of(float cmin, float amax, bool prune) {
    if (!prune) return kInf;
    if (!(cmin < kInf)) return -kInf;
    const float d = fmaxf((amax + cmin) * 0x1p-20f, 0x1p-126f);
    return cmin + d;
}

template <int R, int KL, int NHS>
__global__ __launch_bounds__(kS2Threads) void spec2_kernel(Spec2Model m, Spec2Batch b) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t n = m.n, H = m.H, NH = m.NH;
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t q = blockIdx.x;
    const Spec2Lds L = spec2_lds_layout(n, KL, NH, H);
    float* vl = lds + L.v;
    float2* LP = reinterpret_cast<float2*>(lds + L.lp);
    float2* HP = reinterpret_cast<float2*>(lds + L.hp);
    uint16_t* CL = reinterpret_cast<uint16_t*>(lds + L.cl);
    uint32_t* hacc = reinterpret_cast<uint32_t*>(lds + L.hacc);
    uint32_t* cmin = reinterpret_cast<uint32_t*>(lds + L.cmin);  // [2][H] keys
    uint32_t* ccnt = reinterpret_cast<uint32_t*>(lds + L.ccnt);  // [2][H]
    float* EH = lds + L.eh;                                      // [2 parity][2 (s1, s2)][H]
    uint32_t* hoff = reinterpret_cast<uint32_t*>(lds + L.hoff);  // [H + 1]
    float* amax = lds + L.amax;                                  // [H]

    const uint32_t nch = b.nchunks[q];
    float* vg = b.v + (size_t)q * n;
    const uint8_t* sym = b.symbols + b.sym_off[q];
    const uint32_t len = b.len[q];
    const bool prune = m.prune != 0;

    for (uint32_t j = t; j < n; j += kS2Threads) vl[j] = vg[j];
    for (uint32_t h = t; h < H; h += kS2Threads) {
        hoff[h] = m.hoff[h];
        amax[h] = m.amax[h];
        cmin[h] = cmin[H + h] = okey(kInf);
        ccnt[h] = ccnt[H + h] = 0;
    }
    if (t == 0) hoff[H] = m.hoff[H];

    // the thread's light rows r = s * 1024 + t: terms (packed m | (heavy index of m + 1) << 16)
    uint32_t lc[R][KL];
    float lv[R][KL];
#pragma unroll
    for (int s = 0; s < R; ++s)
#pragma unroll
        for (int k = 0; k < KL; ++k) {
            lc[s][k] = m.lcol[((size_t)s * KL + k) * kS2Threads + t];
            lv[s][k] = m.lval[((size_t)s * KL + k) * kS2Threads + t];
        }
    // the thread's heavy terms x = hs * 1024 + t (sorted by row), their row's heavy index
    uint32_t hc[NHS], hh[NHS];
    float hv[NHS];
    uint32_t uni = 0;  // bit hs: the wave's 64 terms of slot hs all belong to one heavy row
#pragma unroll
    for (int hs = 0; hs < NHS; ++hs) {
        hc[hs] = m.hcol[(size_t)hs * kS2Threads + t];
        hv[hs] = m.hval[(size_t)hs * kS2Threads + t];
        hh[hs] = m.hhid[(size_t)hs * kS2Threads + t];
        const uint32_t h0 = (uint32_t)__builtin_amdgcn_readlane((int)hh[hs], 0);
        const uint32_t h63 = (uint32_t)__builtin_amdgcn_readlane((int)hh[hs], 63);
        if (h0 == h63 && h0 < H) uni |= 1u << hs;
    }
    const uint32_t hrow_t = t < H ? m.hrow[t] : 0;  // H <= kS2Threads (host check)

    // symbols in per-wave VGPR windows: lane l holds bytes wbase + 4l .. +3 (256 per window)
    auto load_win = [&](uint32_t base) -> uint32_t {
        const uint32_t off = base + 4 * lane;
        return off + 4 <= len + kSymPad ? *reinterpret_cast<const uint32_t*>(sym + off) : 0u;
    };
    uint32_t wbase = 0, wcur = load_win(0), wnext = load_win(256);
    auto sym_at = [&](uint32_t i) -> uint32_t {  // i >= wbase (uniform)
        const uint32_t off = i - wbase;
        const uint32_t word = off < 256 ? (uint32_t)__builtin_amdgcn_readlane((int)wcur, (int)(off >> 2))
                                        : (uint32_t)__builtin_amdgcn_readlane((int)wnext, (int)((off - 256) >> 2));
        return (word >> ((off & 3u) * 8)) & 0xFFu;
    };
    auto advance_win = [&](uint32_t i) {  // keep i (and i + 3) inside the two windows
        if (i >= wbase + 256) {
            wbase += 256;
            wcur = wnext;
            wnext = load_win(wbase + 256);
        }
    };

    // E of the thread's light rows for the current chunk (e1, e2) and the next (n1, n2)
    float e1[R], e2[R], n1[R], n2[R];
    float hn1 = kInf, hn2 = kInf;  // t < H: E of heavy row t for the next chunk
    auto fetch_e = [&](uint32_t c, float (&f1)[R], float (&f2)[R], float& g1, float& g2) {
        const uint32_t s1 = sym_at(1 + 2 * c), s2 = sym_at(2 + 2 * c);
        const float* E1 = m.emis + (size_t)s1 * n;
        const float* E2 = m.emis + (size_t)s2 * n;
#pragma unroll
        for (int s = 0; s < R; ++s) {
            const uint32_t r = s * kS2Threads + t;
            f1[s] = r < n ? E1[r] : kInf;
            f2[s] = r < n ? E2[r] : kInf;
        }
        if (t < H) {
            g1 = E1[hrow_t];
            g2 = E2[hrow_t];
        }
    };
    if (nch) {
        fetch_e(0, e1, e2, hn1, hn2);
        if (t < H) {
            EH[t] = hn1;
            EH[H + t] = hn2;
        }
    }
    __syncthreads();
    for (uint32_t h = t; h < H; h += kS2Threads) hacc[h] = okey(vl[m.hrow[h]]);
    __syncthreads();

    auto vread = [&](uint32_t c) -> float {  // score of the packed column c (light: vl, heavy: hacc)
        const uint32_t mh = c >> 16;
        return mh ? okey_val(hacc[mh - 1]) : vl[c & 0xFFFFu];
    };
    // min over p's terms of fl(fl(a + b) + v): light p from LP, heavy p from its candidates
    auto inner = [&](uint32_t pc, float a, uint32_t par) -> float {
        float acc = kInf;
        const uint32_t ph = pc >> 16;
        if (ph == 0) {
            const uint32_t p = pc & 0xFFFFu;
            if constexpr (KL == 2) {
                const float4 pr = *reinterpret_cast<const float4*>(LP + (size_t)p * 2);
                acc = fminf((a + pr.x) + pr.y, (a + pr.z) + pr.w);
            } else {
#pragma unroll
                for (int k = 0; k < KL; k += 2) {
                    const float4 pr = *reinterpret_cast<const float4*>(LP + (size_t)p * KL + k);
                    acc = fminf(acc, fminf((a + pr.x) + pr.y, (a + pr.z) + pr.w));
                }
            }
        } else {
            const uint32_t h = ph - 1;
            const uint32_t cnt = ccnt[par * H + h], base = hoff[h];
            for (uint32_t i = 0; i < cnt; ++i) {
                const float2 pr = HP[CL[base + i]];
                acc = fminf(acc, (a + pr.x) + pr.y);
            }
        }
        return acc;
    };

    float cv[NHS];
    for (uint32_t c = 0; c < nch; ++c) {
        // opaque per iteration: the addresses derived from the terms are recomputed in the chunk
        // (a few VALU) instead of being hoisted out of the loop into ~100 more VGPRs (spills)
#pragma unroll
        for (int s = 0; s < R; ++s)
#pragma unroll
            for (int k = 0; k < KL; ++k) asm volatile("" : "+v"(lc[s][k]));
#pragma unroll
        for (int hs = 0; hs < NHS; ++hs) asm volatile("" : "+v"(hc[hs]), "+v"(hh[hs]));
        const uint32_t par = c & 1u;
        const float* EHc = EH + par * 2 * H;
        const bool more = c + 1 < nch;
        if (more) {
            advance_win(2 * c + 3);
            fetch_e(c + 1, n1, n2, hn1, hn2);
        }
        // ---- phase 1: (b, v_m) pairs; heavy c_f and its per-row minimum
#pragma unroll
        for (int s = 0; s < R; ++s) {
            const uint32_t r = s * kS2Threads + t;
            if (r < n) {
#pragma unroll
                for (int k = 0; k < KL; ++k) {
                    const uint32_t cc = lc[s][k];
                    LP[(size_t)r * KL + k] = cc == kNone ? make_float2(kInf, kInf)
                                                         : make_float2(e1[s] + lv[s][k], vread(cc));
                }
            }
        }
#pragma unroll
        for (int hs = 0; hs < NHS; ++hs) {
            cv[hs] = kInf;
            if (hs * kS2Threads + w * 64 >= NH) continue;  // wave-uniform
            const uint32_t x = hs * kS2Threads + t;
            const bool ok = x < NH;
            if (ok) {
                const float bb = EHc[hh[hs]] + hv[hs];
                const float vm = vread(hc[hs]);
                HP[x] = make_float2(bb, vm);
                cv[hs] = bb + vm;
            }
            if (uni & (1u << hs)) {
                const float r = wave_min63(cv[hs]);
                if (lane == 63) lds_min_u32(cmin + par * H + hh[hs], okey(r));
            } else if (ok) {
                lds_min_u32(cmin + par * H + hh[hs], okey(cv[hs]));
            }
        }
        __syncthreads();
        // ---- phase 1b: candidates; next chunk's heavy E; resets for the next chunk
#pragma unroll
        for (int hs = 0; hs < NHS; ++hs) {
            if (hs * kS2Threads + w * 64 >= NH) continue;
            const uint32_t x = hs * kS2Threads + t;
            const bool ok = x < NH;
            const uint32_t h = ok ? hh[hs] : 0;
            const bool cand = ok && cv[hs] <= theta_of(okey_val(cmin[par * H + h]), amax[h], prune);
            if (uni & (1u << hs)) {
                const uint64_t bal = __builtin_amdgcn_ballot_w64(cand);
                if (bal) {
                    uint32_t base = 0;
                    if (lane == 0)
                        base = __hip_atomic_fetch_add(ccnt + par * H + h, (uint32_t)__builtin_popcountll(bal),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
                    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                    if (cand) CL[hoff[h] + base + below] = (uint16_t)x;
                }
            } else if (cand) {
                const uint32_t pos = __hip_atomic_fetch_add(ccnt + par * H + h, 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_WORKGROUP);
                CL[hoff[h] + pos] = (uint16_t)x;
            }
        }
        if (t < H) {
            hacc[t] = okey(kInf);
            cmin[(par ^ 1u) * H + t] = okey(kInf);
            ccnt[(par ^ 1u) * H + t] = 0;
            if (more) {
                EH[(par ^ 1u) * 2 * H + t] = hn1;
                EH[(par ^ 1u) * 2 * H + H + t] = hn2;
            }
        }
        __syncthreads();
        // ---- phase 2: the chunk's products applied to v
#pragma unroll
        for (int s = 0; s < R; ++s) {
            const uint32_t r = s * kS2Threads + t;
            if (r < n) {
                float acc = kInf;
#pragma unroll
                for (int k = 0; k < KL; ++k) {
                    const uint32_t cc = lc[s][k];
                    if (cc != kNone) acc = fminf(acc, inner(cc, e2[s] + lv[s][k], par));
                }
                vl[r] = acc;  // heavy rows' entries are unused (their scores live in hacc)
            }
        }
#pragma unroll
        for (int hs = 0; hs < NHS; ++hs) {
            if (hs * kS2Threads + w * 64 >= NH) continue;
            const uint32_t x = hs * kS2Threads + t;
            const bool ok = x < NH;
            float acc = kInf;
            if (ok) acc = inner(hc[hs], EHc[H + hh[hs]] + hv[hs], par);
            if (uni & (1u << hs)) {
                const float r = wave_min63(acc);
                if (lane == 63) lds_min_u32(hacc + hh[hs], okey(r));
            } else if (ok) {
                lds_min_u32(hacc + hh[hs], okey(acc));
            }
        }
        __syncthreads();
        if (more) {
#pragma unroll
            for (int s = 0; s < R; ++s) {
                e1[s] = n1[s];
                e2[s] = n2[s];
            }
        }
    }
    for (uint32_t h = t; h < H; h += kS2Threads) vl[m.hrow[h]] = okey_val(hacc[h]);
    __syncthreads();
    for (uint32_t j = t; j < n; j += kS2Threads) vg[j] = vl[j];
}

template <int R, int KL, int NHS>
const void* spec2_ptr() {
    return reinterpret_cast<const void*>(&spec2_kernel<R, KL, NHS>);
}

const void* spec2_kernel_for(uint32_t R, uint32_t KL, uint32_t NHS) {
    const uint32_t r = R <= 2 ? 2 : R <= 4 ? 4 : 0;
    const uint32_t k = KL <= 2 ? 2 : KL <= 4 ? 4 : 0;
    const uint32_t h = NHS <= 4 ? 4 : NHS <= 8 ? 8 : 0;
    switch (r * 100 + k * 10 + h) {
        case 224: return spec2_ptr<2, 2, 4>();
        case 228: return spec2_ptr<2, 2, 8>();
        case 244: return spec2_ptr<2, 4, 4>();
        case 248: return spec2_ptr<2, 4, 8>();
        case 424: return spec2_ptr<4, 2, 4>();
        case 428: return spec2_ptr<4, 2, 8>();
        case 444: return spec2_ptr<4, 4, 4>();
        case 448: return spec2_ptr<4, 4, 8>();
        default: return nullptr;
    }
}

}  // namespace

uint32_t spec2_round_r(uint32_t R) { return R <= 2 ? 2 : R <= 4 ? 4 : 0; }
uint32_t spec2_round_kl(uint32_t KL) { return KL <= 2 ? 2 : KL <= 4 ? 4 : 0; }
uint32_t spec2_round_nhs(uint32_t NHS) { return NHS <= 4 ? 4 : NHS <= 8 ? 8 : 0; }

hipError_t launch_spec2(const Spec2Model& m, const Spec2Batch& b, hipStream_t stream) {
    const void* fn = spec2_kernel_for(m.R, m.KL, m.NHS);
    if (!fn || m.H > kS2Threads || m.n > 65535 || m.NH > 65535 || m.R != spec2_round_r(m.R) ||
        m.KL != spec2_round_kl(m.KL) || m.NHS != spec2_round_nhs(m.NHS) || m.n > m.R * kS2Threads ||
        m.NH > m.NHS * kS2Threads)
        return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    const size_t lds = spec2_lds_layout(m.n, m.KL, m.NH, m.H).bytes;
    if (lds > kMaxLdsBytes) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    Spec2Model mm = m;
    Spec2Batch bb = b;
    void* args[] = {&mm, &bb};
    return hipLaunchKernel(fn, dim3(b.nseq), dim3(kS2Threads), args, lds, stream);
}

}  // namespace svh
