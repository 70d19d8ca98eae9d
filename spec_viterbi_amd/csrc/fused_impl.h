// Fused persistent Viterbi step kernel (gfx950).  Included by fused_r*.hip, one family per file.
//
// Reference hot loop: Viterbi_impl/GraphBLAS_impl.cpp:59-73 (and the bit-identical level-1 _spec
// tail, GraphBLAS_spec_impl.cpp:84-89):
//     v'[j] = min_k fl( fl(E[o][j] + T^T[j][k]) + v[k] )
//
// One workgroup walks every observation of one sequence.  Per workgroup:
//   * T^T lives in VGPRs for the whole launch.  State j is owned by thread j % B, slot j / B.
//     LIGHT rows (<= R terms) are evaluated by their owner from LDS gathers; HEAVY rows (the MSV
//     N and C states, in-degree n-1) are reduced over every thread's own sources, DPP-min across
//     the wave and one LDS atomic-min per wave into the row's heavy slot.
//   * v is triple-buffered in LDS (read i-1, write i, reset heavy slots of i+1) so one barrier per
//     observation suffices.  Each buffer: [v_0 .. v_{est-1} | +inf scratch | heavy slots | pad].
//   * Emission rows E[o] stream into a 3-slot LDS ring by global_load_lds_dwordx4 (LDS-DMA), one
//     observation ahead, in flight across the barrier (counted vmcnt, raw s_barrier); symbols are
//     staged in LDS in chunks.  The loop issues no other vector-memory loads.
//   * MODE_UNI (MSV-like heavy rows: one dominant weight w_h over a source set U shared by all
//     heavy rows, plus <= XM exception terms):  min_{k in U} fl(a + v[k]) == fl(a + min_{k in U}
//     v[k]) for a = fl(E_h + w_h) because fp32 addition is monotone, so U costs one min per
//     term, shared by every heavy row.  Bit-identical to the term-by-term form.
//   * PATHS: per-step argmin backpointers (lowest predecessor index on ties) as uint16.
#pragma once

#include "device_common.h"
#include "kernels.h"

namespace svh {

template <int SM, int R, int HM, int XM, int MODE, bool PATHS>
__global__ __launch_bounds__(kMaxFusedThreads) void fused_viterbi_kernel(FusedModel m,
                                                                         FusedBatch b) {
    using namespace dev;
    static_assert(!(PATHS && MODE == kHeavyUniform), "argmin ties need the term-by-term form");
    static_assert(XM <= kMaxExc, "exception capacity");
    constexpr int NDMA = (SM + 3) / 4;  // 16-byte LDS-DMA instructions per thread per E row
    extern __shared__ __attribute__((aligned(16))) float lds[];

    // ---- loop invariants into registers (kernel-argument memory would be re-read after every
    //      barrier's memory clobber) -----------------------------------------------------------
    const uint32_t B = m.B, n = m.n, est = m.estride, vstride = m.vstride, H = m.H;
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6, q = blockIdx.x;
    const uint32_t scratch = est;  // always +inf
    const uint32_t hs0 = est + 1;  // heavy slots hs0 .. hs0+HM-1
    const float* __restrict__ emis = m.emis;
    int hrow[HM];
    float hw[HM];
    uint32_t xk[HM][XM];
    float xw[HM][XM];
#pragma unroll
    for (int h = 0; h < HM; ++h) {
        hrow[h] = m.hrow[h];
        hw[h] = m.hw[h];
#pragma unroll
        for (int x = 0; x < XM; ++x) {
            xk[h][x] = m.xk[h][x];
            xw[h][x] = m.xw[h][x];
        }
    }

    const uint32_t eslot = NDMA * B * 4;  // floats per E-ring slot
    float* vbuf[3] = {lds, lds + vstride, lds + 2 * vstride};
    float* ering = lds + 3 * vstride;
    uint64_t* kbuf = reinterpret_cast<uint64_t*>(ering + 3 * eslot);  // [3][HM] (PATHS)
    float* red = reinterpret_cast<float*>(kbuf + 3 * HM);              // [2][kMaxWaves]
    uint32_t* symr = reinterpret_cast<uint32_t*>(red + 2 * kMaxWaves);  // kSymChunk + 64 bytes

    // ---- register-resident schedule ------------------------------------------------------
    float lv[SM][R];
    uint32_t lc[SM][R];
#pragma unroll
    for (int s = 0; s < SM; ++s)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t idx = ((size_t)s * R + r) * B + t;
            lc[s][r] = m.lcol[idx];
            lv[s][r] = m.lval[idx];
        }
    constexpr int HV = (MODE == kHeavyGeneral) ? HM : 1;
    float hv[HV][SM];
    uint32_t hk[HV][SM];
    float hz[SM];
#pragma unroll
    for (int s = 0; s < SM; ++s) {
        if constexpr (MODE == kHeavyUniform) {
            hz[s] = m.hmask[(size_t)s * B + t];
        } else {
            hz[s] = 0.0f;
#pragma unroll
            for (int h = 0; h < HM; ++h) {
                const size_t idx = ((size_t)h * SM + s) * B + t;
                hv[h][s] = m.hval[idx];
                if constexpr (PATHS) hk[h][s] = m.hvalid[idx] ? (uint32_t)(s * B + t) : 0xFFFFFFFFu;
                else hk[h][s] = 0;
            }
        }
    }

    // ---- sequence setup --------------------------------------------------------------------
    const uint8_t* sym = b.symbols + b.sym_off[q];
    const uint32_t len = b.end[q];
    uint32_t i = b.begin[q];
    const bool fresh = (i == 0);
    uint32_t sbase = fresh ? 0u : (i & ~3u);
    auto stage_symbols = [&](uint32_t from) {
        // Each sequence is 16-byte aligned and followed by >= kSymPad zero bytes (host side of
        // the boundary), so words up to len + kSymPad are readable and decode to symbol 0.
        const uint32_t* src = reinterpret_cast<const uint32_t*>(sym + from);
        const uint32_t avail = (len + kSymPad - from) / 4;
        const uint32_t words = min((uint32_t)(kSymChunk + 64) / 4, avail);
        for (uint32_t x = t; x < words; x += B) symr[x] = src[x];
    };
    stage_symbols(sbase);
    auto sym_at = [&](uint32_t idx) -> uint32_t {
        return reinterpret_cast<const uint8_t*>(symr)[idx - sbase];
    };
    // E row of symbol o -> ring slot (LDS-DMA, 16 B per lane, wave-linear destination)
    auto dma_e = [&](uint32_t o, float* slot) {
        const float* row = emis + (size_t)o * est;
#pragma unroll
        for (int c = 0; c < NDMA; ++c) {
            const uint32_t base = (c * B + wave * 64u) * 4u;  // floats
            lds_dma16(row + base + lane * 4u, uniform(lds_addr(slot + base)));
        }
    };

    {
        const float* e0 = emis + (size_t)sym[0] * est;
        const float* vin = fresh ? nullptr : b.v_in + (size_t)b.v_in_row[q] * n;
        float* v0 = vbuf[0];
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            const uint32_t j = s * B + t;
            if (fresh) v0[j] = e0[j] + m.start[j];  // diag(E[s0]) (x) start
            else v0[j] = j < n ? vin[j] : kInf;
        }
        if (t < 3u * (1u + HM)) {
            const uint32_t bsel = t / (1u + HM), slot = t % (1u + HM);  // slot 0: scratch
            float val = kInf;
            if (bsel == 0 && slot > 0 && slot - 1 < H) {
                const int hr = hrow[slot - 1];
                val = fresh ? e0[hr] + m.start[hr] : vin[hr];
            }
            vbuf[bsel][scratch + slot] = val;
            if constexpr (PATHS) {
                if (slot > 0)
                    kbuf[bsel * HM + slot - 1] =
                        (bsel == 0 && slot - 1 < H) ? lex_key(val, 0xFFFFFFFFu) : ~0ull;
            }
        }
    }
    if (fresh) i = 1;
    __syncthreads();  // symbols staged, v0 written
    if (i < len) {
        dma_e(uniform(sym_at(i)), ering);
        dma_e(uniform(sym_at(i + 1)), ering + eslot);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    uint16_t* bp = PATHS ? b.bp + b.bp_off[q] : nullptr;

    // ---- one observation -----------------------------------------------------------------
    //   vc/ec: scores and E row of observation i (read), vn: scores written, vr: buffer of i+1
    //   (heavy slots reset here), enext2: ring slot filled for observation i+2.
    auto step = [&](const float* vc, float* vn, float* vr, uint64_t* kc, uint64_t* kn,
                    uint64_t* kr, float* vcw, const float* ecur, float* enext2) {
        if (i + 3 >= sbase + kSymChunk) {  // uniform: refill the symbol ring (rare)
            sbase = i & ~3u;
            __syncthreads();
            stage_symbols(sbase);
            __syncthreads();
        }
        const uint32_t o2 = sym_at(i + 2);  // consumed by the DMA at the end of the step

        if constexpr (PATHS) {
            // publish last step's heavy values into this wave's view of v; backpointers of
            // heavy rows for observation i-1
            if (lane == 0) {
#pragma unroll
                for (int h = 0; h < HM; ++h) vcw[hs0 + h] = lex_key_value(kc[h]);
            }
            if (t == 0 && i >= 2) {
#pragma unroll
                for (int h = 0; h < HM; ++h) {
                    if ((uint32_t)h < H) {
                        const uint32_t k = lex_key_index(kc[h]);
                        bp[(size_t)(i - 2) * n + hrow[h]] = (uint16_t)(k == 0xFFFFFFFFu ? kNoPred : k);
                    }
                }
            }
        }

        // ---- all LDS reads of the step first (they cannot be proven disjoint from the writes)
        float vs[SM], ec[SM], g[SM][R], ehc[HM], gx[HM][XM];
#pragma unroll
        for (int s = 0; s < SM; ++s) vs[s] = vc[s * B + t];
#pragma unroll
        for (int s = 0; s < SM; ++s) ec[s] = ecur[s * B + t];
#pragma unroll
        for (int s = 0; s < SM; ++s)
#pragma unroll
            for (int r = 0; r < R; ++r) g[s][r] = vc[lc[s][r]];
#pragma unroll
        for (int h = 0; h < HM; ++h) {
            ehc[h] = ecur[hrow[h]];
#pragma unroll
            for (int x = 0; x < XM; ++x) gx[h][x] = vc[xk[h][x]];
        }

        // ---- heavy rows
        if constexpr (MODE == kHeavyUniform) {
            float mu = kInf;
#pragma unroll
            for (int s = 0; s < SM; ++s) mu = fminf(mu, vs[s] + hz[s]);
            mu = wave_min63(mu);
            if (lane == 63) {
#pragma unroll
                for (int h = 0; h < HM; ++h) {
                    float a = (ehc[h] + hw[h]) + mu;
#pragma unroll
                    for (int x = 0; x < XM; ++x) a = fminf(a, (ehc[h] + xw[h][x]) + gx[h][x]);
                    lds_atomic_min(&vn[hs0 + h], a);
                }
            }
        } else if constexpr (!PATHS) {
            float acc[HM];
#pragma unroll
            for (int h = 0; h < HM; ++h) {
                acc[h] = kInf;
#pragma unroll
                for (int s = 0; s < SM; ++s) acc[h] = fminf(acc[h], (ehc[h] + hv[h][s]) + vs[s]);
            }
#pragma unroll
            for (int h = 0; h + 1 < HM; h += 2) wave_min63x2(acc[h], acc[h + 1]);
            if constexpr (HM % 2) acc[HM - 1] = wave_min63(acc[HM - 1]);
            if (lane == 63) {
#pragma unroll
                for (int h = 0; h < HM; ++h) {
                    float a = acc[h];
#pragma unroll
                    for (int x = 0; x < XM; ++x) a = fminf(a, (ehc[h] + xw[h][x]) + gx[h][x]);
                    lds_atomic_min(&vn[hs0 + h], a);
                }
            }
        } else {
#pragma unroll
            for (int h = 0; h < HM; ++h) {
                float acc = kInf;
                uint32_t ak = 0xFFFFFFFFu;
#pragma unroll
                for (int s = 0; s < SM; ++s) lex_min(acc, ak, (ehc[h] + hv[h][s]) + vs[s], hk[h][s]);
                wave_lexmin63(acc, ak);
#pragma unroll
                for (int x = 0; x < XM; ++x) {
                    const uint32_t src = xk[h][x];
                    const uint32_t kx = src == scratch ? 0xFFFFFFFFu
                                        : (src >= hs0 ? (uint32_t)hrow[src - hs0] : src);
                    lex_min(acc, ak, (ehc[h] + xw[h][x]) + gx[h][x], kx);
                }
                if (lane == 63) lds_atomic_min(&kn[h], lex_key(acc, ak));
            }
        }

        // ---- light rows: emission masking fused with the (min,+) product
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            const float e = ec[s];
            const uint32_t j = s * B + t;
            if constexpr (!PATHS) {
                float r = kInf;
#pragma unroll
                for (int k = 0; k < R; ++k) r = fminf(r, (e + lv[s][k]) + g[s][k]);
                vn[j] = r;
            } else {
                float r = kInf;
                uint32_t rk = 0xFFFFFFFFu;
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const uint32_t src = lc[s][k];
                    const uint32_t kx = src == scratch ? 0xFFFFFFFFu
                                        : (src >= hs0 ? (uint32_t)hrow[src - hs0] : src);
                    lex_min(r, rk, (e + lv[s][k]) + g[s][k], kx);
                }
                vn[j] = r;
                if (j < n) bp[(size_t)(i - 1) * n + j] = (uint16_t)(rk == 0xFFFFFFFFu ? kNoPred : rk);
            }
        }

        // reset heavy slots of the buffer written at i+1 (last read at i-1)
        if (t < (uint32_t)HM) {
            vr[hs0 + t] = kInf;
            if constexpr (PATHS) kr[t] = ~0ull;
        }

        // stream the E row of observation i+2; keep it in flight across the barrier, retire
        // the one issued last step (all older vector-memory ops included)
        dma_e(uniform(o2), enext2);
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(NDMA)
                     : "memory");
    };

    // ---- main loop: three observations per iteration (fixed buffer roles) ----------------
    uint32_t cur = 0;
    float* const e0s = ering;
    float* const e1s = ering + eslot;
    float* const e2s = ering + 2 * eslot;
    while (true) {
        if (i >= len) { cur = 0; break; }
        step(vbuf[0], vbuf[1], vbuf[2], kbuf, kbuf + HM, kbuf + 2 * HM, vbuf[0], e0s, e2s);
        if (++i >= len) { cur = 1; break; }
        step(vbuf[1], vbuf[2], vbuf[0], kbuf + HM, kbuf + 2 * HM, kbuf, vbuf[1], e1s, e0s);
        if (++i >= len) { cur = 2; break; }
        step(vbuf[2], vbuf[0], vbuf[1], kbuf + 2 * HM, kbuf, kbuf + HM, vbuf[2], e2s, e1s);
        ++i;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- epilogue -------------------------------------------------------------------------
    float* vc = vbuf[cur];
    if (t < H) {
        float val = vc[hs0 + t];
        if constexpr (PATHS) {
            const uint64_t key = kbuf[cur * HM + t];
            val = lex_key_value(key);
            if (len >= 2) {
                const uint32_t k = lex_key_index(key);
                bp[(size_t)(len - 2) * n + hrow[t]] = (uint16_t)(k == 0xFFFFFFFFu ? kNoPred : k);
            }
        }
        vc[hrow[t]] = val;
    }
    __syncthreads();
    float* out = b.scores + (size_t)q * n;
    float bv = kInf;
    uint32_t bk = 0xFFFFFFFFu;
#pragma unroll
    for (int s = 0; s < SM; ++s) {
        const uint32_t j = s * B + t;
        if (j < n) {
            const float x = vc[j];
            out[j] = x;
            lex_min(bv, bk, x, j);
        }
    }
    // block argmin (lowest index of the minimum final score)
    wave_lexmin63(bv, bk);
    uint32_t* redk = reinterpret_cast<uint32_t*>(red + kMaxWaves);
    if (lane == 63) {
        red[wave] = bv;
        redk[wave] = bk;
    }
    __syncthreads();
    if (t == 0 && b.best) {
        float fv = red[0];
        uint32_t fk = redk[0];
        for (uint32_t w = 1; w < (B >> 6); ++w) lex_min(fv, fk, red[w], redk[w]);
        b.best[q] = (fk == 0xFFFFFFFFu) ? -1 : (int64_t)fk;
    }
}

// Kernel pointer for (SM, PATHS) of one family.
template <int R, int HM, int XM, int MODE, bool P>
const void* fused_family_ptr(int smax) {
    switch (smax) {
#define SVH_CASE(SMV) \
    case SMV: return reinterpret_cast<const void*>(&fused_viterbi_kernel<SMV, R, HM, XM, MODE, P>);
        SVH_CASE(1) SVH_CASE(2) SVH_CASE(3) SVH_CASE(4) SVH_CASE(5) SVH_CASE(6) SVH_CASE(8)
        SVH_CASE(10) SVH_CASE(12) SVH_CASE(16)
#undef SVH_CASE
        default: return nullptr;
    }
}

}  // namespace svh
