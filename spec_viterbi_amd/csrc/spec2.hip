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
// Data on chip: the scores of the light rows (vl) and of the heavy rows (hacc: order-preserving
// keys, so the per-row minima are ds_min_u32); one array of (b, v_m) pairs: per light row p its KL
// terms' pairs (LP), per heavy row its candidates (CP).  Every term carries two precomputed words:
// where its column's score is read (phase 1) and where its column's pair list starts plus the
// cell holding that list's length (phase 2: KL for a light column, the candidate count for a heavy
// one, 0 for a padding term), so no step branches on the kind of a column.
// Per chunk (symbols s1 = seq[1+2c], s2 = seq[2+2c]), three barriers (LDS only: the next chunk's
// emission loads stay in flight across them):
//   1  light rows p: LP[p][k] = (fl(E_s1[p] + T^T[p][m_k]), v[m_k]); heavy terms of row p: (b, v_m)
//      in registers, c_f = fl(b + v_m), the row's minimum c_f (one wave reduction + LDS atomic);
//   1b heavy terms: the candidates' pairs (c_f <= theta) appended to CP[row];
//   2  light rows j: v'[j] = min over its terms p of the loop over p's pairs; heavy terms (j, p):
//      the same per term, then the row's minimum into hacc[j].
#include "device_common.h"
#include "kernels.h"

namespace svh {

using namespace dev;

namespace {

constexpr uint32_t kS2Threads = kSpec2Threads;

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

// Diagnostics (-DSVH_SPEC2_DIAG, then SVH_SPEC2_DEBUG=1): shader cycles per wave spent in phase 1,
// the barrier after it, phase 1b, its barrier, phase 2, its barrier, and the whole loop.
#ifdef SVH_SPEC2_DIAG
#define S2_T(k)                                                     \
    do {                                                            \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(); \
        dg[k] += t1 - t0;                                           \
        t0 = t1;                                                    \
    } while (0)
#else
#define S2_T(k) ((void)0)
#endif

template <int R, int KL, int NHS>
__global__ __launch_bounds__(kS2Threads) void spec2_kernel(Spec2Model m, Spec2Batch b) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t n = m.n, H = m.H, nhs = m.nhs;
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t q = blockIdx.x;
    if (b.run_mask && b.run_mask[q] == 0) return;  // a fallback pass: only the flagged rows
    const Spec2Lds L = spec2_lds_layout(n, KL, m.NP, H);
    float* vl = lds + L.v;                                       // [n + 1]: vl[n] = +inf
    float2* PR = reinterpret_cast<float2*>(lds + L.pairs);       // LP [n][KL] | CP [NP]
    uint32_t* hacc = reinterpret_cast<uint32_t*>(lds + L.hacc);  // [H + 1] keys (H: padding row)
    uint32_t* cmin = reinterpret_cast<uint32_t*>(lds + L.cmin);  // [2][H + 1] keys
    uint32_t* ccnt = reinterpret_cast<uint32_t*>(lds + L.ccnt);  // [2][H + 2]: H = KL, H + 1 = 0
    float* EH = lds + L.eh;                                      // [2 parity][2 (s1, s2)][H + 1]
    float* amax = lds + L.amax;                                  // [H + 1]
    const uint32_t H1 = H + 1, H2 = H + 2;

    const uint32_t nch = b.nchunks[q];
    float* vg = b.v + (size_t)q * n;
    const uint8_t* sym = b.symbols + b.sym_off[q];
    const uint32_t len = b.len[q];
    const bool prune = m.prune != 0;

    for (uint32_t j = t; j < n; j += kS2Threads) vl[j] = vg[j];
    if (t == 0) vl[n] = kInf;
    for (uint32_t h = t; h <= H; h += kS2Threads) {
        amax[h] = h < H ? m.amax[h] : 0.0f;
        cmin[h] = cmin[H1 + h] = okey(kInf);
        hacc[h] = okey(h < H ? vg[m.hrow[h]] : kInf);
        EH[h] = EH[H1 + h] = EH[2 * H1 + h] = EH[3 * H1 + h] = kInf;
    }
    for (uint32_t h = t; h < H2; h += kS2Threads) ccnt[h] = ccnt[H2 + h] = h == H ? (uint32_t)KL : 0u;

    // light rows r = s * 1024 + t: per term the score address (la), the pair list (lb: base | cell
    // << 20) and T^T's value
    uint32_t la[R][KL], lb[R][KL];
    float lv[R][KL];
#pragma unroll
    for (int s = 0; s < R; ++s)
#pragma unroll
        for (int k = 0; k < KL; ++k) {
            const size_t i = ((size_t)s * KL + k) * kS2Threads + t;
            la[s][k] = m.la[i];
            lb[s][k] = m.lb[i];
            lv[s][k] = m.lv[i];
        }
    // heavy terms: this thread's row (H: none) and its nhs terms (the row's terms padded to a
    // multiple of nhs, so a thread's terms never straddle two rows)
    const uint32_t hr = m.thr[t];
    const uint32_t hcp = m.tcp[t];  // the row's CP range (pair index)
    uint32_t ha[NHS], hb[NHS];
    float hv[NHS];
#pragma unroll
    for (int hs = 0; hs < NHS; ++hs) {
        const size_t i = (size_t)t * NHS + hs;
        ha[hs] = m.ha[i];
        hb[hs] = m.hb[i];
        hv[hs] = m.hv[i];
    }
    const uint32_t hr0 = (uint32_t)__builtin_amdgcn_readlane((int)hr, 0);
    const uint32_t hr63 = (uint32_t)__builtin_amdgcn_readlane((int)hr, 63);
    const bool hwave = __builtin_amdgcn_ballot_w64(hr < H) != 0;  // the wave has heavy terms
    const bool huni = hr0 == hr63 && hr0 < H;                     // ... all of one row
    const uint32_t hrow_t = t < H ? m.hrow[t] : 0;                // H <= kS2Threads - 2 (host check)

    // symbols in per-wave VGPR windows: lane l holds bytes wbase + 4l .. +3 (256 per window)
    auto load_win = [&](uint32_t base) -> uint32_t {
        const uint32_t off = base + 4 * lane;
        return off + 4 <= len + kSymPad ? *reinterpret_cast<const uint32_t*>(sym + off) : 0u;
    };
    uint32_t wbase = 0, wcur = load_win(0), wnext = load_win(256);
    auto sym_at = [&](uint32_t i) -> uint32_t {  // wbase <= i < wbase + 512 (uniform)
        const uint32_t off = i - wbase;
        const uint32_t word = off < 256 ? (uint32_t)__builtin_amdgcn_readlane((int)wcur, (int)(off >> 2))
                                        : (uint32_t)__builtin_amdgcn_readlane((int)wnext, (int)((off - 256) >> 2));
        return (word >> ((off & 3u) * 8)) & 0xFFu;
    };
    auto advance_win = [&](uint32_t i) {  // keep i and i + 1 inside the two windows
        if (i >= wbase + 256) {
            wbase += 256;
            wcur = wnext;
            wnext = load_win(wbase + 256);
        }
    };

    // E of the thread's light rows for the current chunk (e1, e2) and the next (n1, n2); t < H: E of
    // heavy row t for the next chunk (g1, g2), written to EH at the end of the chunk
    float e1[R], e2[R], n1[R], n2[R];
    float g1 = kInf, g2 = kInf;
    auto fetch_e = [&](uint32_t c, float (&f1)[R], float (&f2)[R]) {
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
        fetch_e(0, e1, e2);
        if (t < H) {
            EH[t] = g1;
            EH[H1 + t] = g2;
        }
    }
    __syncthreads();

    // score of a term's column: light -> vl, heavy -> hacc (a key), padding -> vl[n] = +inf
    auto vread = [&](uint32_t a) -> float {
        const uint32_t raw = __builtin_bit_cast(uint32_t, lds[a & 0x7FFFFFFFu]);
        return (a & 0x80000000u) ? okey_val(raw) : __builtin_bit_cast(float, raw);
    };
    // min over the column's pairs of fl(fl(a + b) + v): a light column's KL pairs with 16-byte
    // reads (no count), a heavy column's candidates (count cell), a padding term none
    auto apply = [&](uint32_t pb, float a, const uint32_t* cc) -> float {
        const uint32_t base = pb & 0xFFFFFu, cell = pb >> 20;
        float acc = kInf;
        if (cell == H) {
#pragma unroll
            for (int k = 0; k < KL; k += 2) {
                const float4 pr = *reinterpret_cast<const float4*>(PR + base + k);
                acc = fminf(acc, fminf((a + pr.x) + pr.y, (a + pr.z) + pr.w));
            }
        } else {
            const uint32_t cnt = cc[cell];
#pragma nounroll
            for (uint32_t i = 0; i < cnt; ++i) {
                const float2 pr = PR[base + i];
                acc = fminf(acc, (a + pr.x) + pr.y);
            }
        }
        return acc;
    };

    float cb[NHS], cm[NHS], cv[NHS];  // heavy terms: (b, v_m) and c_f, phase 1 -> 1b
#ifdef SVH_SPEC2_DIAG
    unsigned long long dg[kSpec2Stamps] = {};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long tloop = t0;
#endif
    for (uint32_t c = 0; c < nch; ++c) {
        // opaque per iteration: what is derived from the term words is recomputed in the chunk
        // instead of being hoisted out of the loop into more VGPRs (spills)
#pragma unroll
        for (int s = 0; s < R; ++s)
#pragma unroll
            for (int k = 0; k < KL; ++k) asm volatile("" : "+v"(la[s][k]), "+v"(lb[s][k]));
#pragma unroll
        for (int hs = 0; hs < NHS; ++hs) asm volatile("" : "+v"(ha[hs]), "+v"(hb[hs]));
        const uint32_t par = c & 1u;
        const float* EHc = EH + par * 2 * H1;
        const uint32_t* ccp = ccnt + par * H2;
        const bool more = c + 1 < nch;
        if (more) {
            advance_win(2 * c + 3);
            fetch_e(c + 1, n1, n2);
        }
        // ---- phase 1: (b, v_m) pairs; heavy c_f and its per-row minimum
#pragma unroll
        for (int s = 0; s < R; ++s) {
            if (s * kS2Threads + w * 64 >= n) continue;  // wave-uniform
            const uint32_t r = s * kS2Threads + t;
            float2 pp[KL];
#pragma unroll
            for (int k = 0; k < KL; ++k) pp[k] = make_float2(e1[s] + lv[s][k], vread(la[s][k]));
            if (r < n) {
#pragma unroll
                for (int k = 0; k < KL; k += 2)
                    *reinterpret_cast<float4*>(PR + (size_t)r * KL + k) = make_float4(pp[k].x, pp[k].y, pp[k + 1].x, pp[k + 1].y);
            }
        }
        if (hwave) {
            const float eh1 = EHc[hr];
            float part = kInf;
#pragma unroll
            for (int hs = 0; hs < NHS; ++hs) {
                cv[hs] = kInf;
                if ((uint32_t)hs >= nhs) continue;  // uniform
                cb[hs] = eh1 + hv[hs];
                cm[hs] = vread(ha[hs]);
                cv[hs] = cb[hs] + cm[hs];
                part = fminf(part, cv[hs]);
            }
            if (huni) {
                part = wave_min63(part);
                if (lane == 63) lds_min_u32(cmin + par * H1 + hr, okey(part));
            } else {
                lds_min_u32(cmin + par * H1 + hr, okey(part));
            }
        }
        S2_T(0);
        lds_barrier();
        S2_T(1);
        // ---- phase 1b: the candidates' pairs; resets for the next chunk
        if (hwave) {
            const float th = theta_of(okey_val(cmin[par * H1 + hr]), amax[hr], prune);
            uint32_t k = 0;
#pragma unroll
            for (int hs = 0; hs < NHS; ++hs)
                if ((uint32_t)hs < nhs) k += (hr < H && cv[hs] <= th) ? 1u : 0u;
            if (__builtin_amdgcn_ballot_w64(k != 0)) {
                if (k) {
                    uint32_t pos = hcp + __hip_atomic_fetch_add(ccnt + par * H2 + hr, k, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
                    for (int hs = 0; hs < NHS; ++hs)
                        if ((uint32_t)hs < nhs && cv[hs] <= th) PR[pos++] = make_float2(cb[hs], cm[hs]);
                }
            }
        }
        for (uint32_t h = t; h < H; h += kS2Threads) {
            hacc[h] = okey(kInf);
            cmin[(par ^ 1u) * H1 + h] = okey(kInf);
            ccnt[(par ^ 1u) * H2 + h] = 0;
        }
        S2_T(2);
        lds_barrier();
        S2_T(3);
        // ---- phase 2: the chunk's products applied to v
#pragma unroll
        for (int s = 0; s < R; ++s) {
            if (s * kS2Threads + w * 64 >= n) continue;
            const uint32_t r = s * kS2Threads + t;
            float acc = kInf;
#pragma unroll
            for (int k = 0; k < KL; ++k) acc = fminf(acc, apply(lb[s][k], e2[s] + lv[s][k], ccp));
            if (r < n) vl[r] = acc;  // heavy rows' entries stay unused (their scores live in hacc)
        }
        if (hwave) {
            const float eh2 = EHc[H1 + hr];
            float part = kInf;
#pragma unroll
            for (int hs = 0; hs < NHS; ++hs)
                if ((uint32_t)hs < nhs) part = fminf(part, apply(hb[hs], eh2 + hv[hs], ccp));
            if (huni) {
                part = wave_min63(part);
                if (lane == 63) lds_min_u32(hacc + hr, okey(part));
            } else if (hr < H) {
                lds_min_u32(hacc + hr, okey(part));
            }
        }
        if (t < H && more) {  // the next chunk's heavy E (loaded at this chunk's start)
            EH[(par ^ 1u) * 2 * H1 + t] = g1;
            EH[(par ^ 1u) * 2 * H1 + H1 + t] = g2;
        }
        S2_T(4);
        lds_barrier();
        S2_T(5);
        if (more) {
#pragma unroll
            for (int s = 0; s < R; ++s) {
                e1[s] = n1[s];
                e2[s] = n2[s];
            }
        }
    }
#ifdef SVH_SPEC2_DIAG
    dg[6] = __builtin_amdgcn_s_memtime() - tloop;
    dg[7] = nch;
    if (m.stamps && lane == 0)
        for (int k = 0; k < kSpec2Stamps; ++k) m.stamps[((size_t)q * 16 + w) * kSpec2Stamps + k] = dg[k];
#endif
    for (uint32_t h = t; h < H; h += kS2Threads) vl[m.hrow[h]] = okey_val(hacc[h]);
    __syncthreads();
    float* vo = b.v_out ? b.v_out + (size_t)q * n : vg;
    for (uint32_t j = t; j < n; j += kS2Threads) vo[j] = vl[j];
}

template <int R, int KL, int NHS>
const void* spec2_ptr() {
    return reinterpret_cast<const void*>(&spec2_kernel<R, KL, NHS>);
}

template <int R, int KL>
const void* spec2_ptr_h(uint32_t NHS) {
    return NHS == 4 ? spec2_ptr<R, KL, 4>() : NHS == 6 ? spec2_ptr<R, KL, 6>() : NHS == 8 ? spec2_ptr<R, KL, 8>() : nullptr;
}

const void* spec2_kernel_for(uint32_t R, uint32_t KL, uint32_t NHS) {
    switch (R * 10 + KL) {
        case 22: return spec2_ptr_h<2, 2>(NHS);
        case 24: return spec2_ptr_h<2, 4>(NHS);
        case 32: return spec2_ptr_h<3, 2>(NHS);
        case 34: return spec2_ptr_h<3, 4>(NHS);
        case 42: return spec2_ptr_h<4, 2>(NHS);
        case 44: return spec2_ptr_h<4, 4>(NHS);
        default: return nullptr;
    }
}

}  // namespace

uint32_t spec2_round_r(uint32_t R) { return R <= 2 ? 2 : R <= 4 ? R : 0; }
uint32_t spec2_round_kl(uint32_t KL) { return KL <= 2 ? 2 : KL <= 4 ? 4 : 0; }
uint32_t spec2_round_nhs(uint32_t NHS) { return NHS <= 4 ? 4 : NHS <= 6 ? 6 : NHS <= 8 ? 8 : 0; }

hipError_t launch_spec2(const Spec2Model& m, const Spec2Batch& b, hipStream_t stream) {
    const void* fn = spec2_kernel_for(m.R, m.KL, m.NHS);
    if (!fn || m.H + 2 > kS2Threads || m.n > 65535 || m.nhs == 0 || m.nhs > m.NHS || m.n > m.R * kS2Threads)
        return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    const size_t lds = spec2_lds_layout(m.n, m.KL, m.NP, m.H).bytes;
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
