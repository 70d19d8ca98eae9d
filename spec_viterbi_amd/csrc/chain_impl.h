// Barrier-free chain Viterbi kernel template (gfx950) for MSV-shaped models (N, M_1..M_L, C; the shape of
// every reference .chmm, chmm_files/silent_hmm_to_chmm.py), emit_num <= 32.
//
// Reference hot loop: Viterbi_impl/GraphBLAS_impl.cpp:59-73 (same association, bit-identical):
//     v'[j] = min_k fl( fl(E[o][j] + T^T[j][k]) + v[k] )
//
// One workgroup per sequence; its waves never meet at an s_barrier inside the loop.
//   * Light scores, the weights of their two terms and the emission table of the thread's own
//     positions for every symbol live in VGPRs (E[o] is picked by the wave-uniform symbol with
//     s_set_gpr_idx), so the loop issues no LDS traffic for them and no vector-memory traffic
//     except one symbol word every four observations.
//   * Position p = t*SM + s is slot s of thread t: the chain predecessor of slot 0 is lane-1's
//     last slot (DPP wave_shr:1); lane 0 takes the previous wave's last value of the previous
//     observation from a tagged LDS word (value | observation tag, one 64-bit word).
//   * Heavy rows: min_{k in U} fl(a + v[k]) == fl(a + min_{k in U} v[k]) (fp32 add is monotone),
//     U = all light rows.  Each wave publishes its partial min of every observation as a tagged
//     word; the heavy scores of observation i-1 are computed (redundantly, in every thread) at
//     observation i from the partials of i-2, so the all-wave exchange has one observation of
//     slack and the waves drift freely by up to two observations.
//   * Rings of 4 tagged words per wave make overwrites safe: a wave at observation i has seen
//     every wave finish observation i-2.  Every spin is bounded (fault word on give-up).
#pragma once

#include <type_traits>

#include "device_common.h"
#include "kernels.h"

namespace svh {

using namespace dev;

namespace {

typedef float f32x32 __attribute__((ext_vector_type(32)));
typedef float f2 __attribute__((ext_vector_type(2)));  // one v_pk_*_f32 operand (aligned VGPR pair)

constexpr uint32_t kRing = kChainRing;  // see the ring argument at the exchange
constexpr uint32_t kSpinLimit = 1u << 22;

// Empty asm that consumes the values: everything computing them is emitted before it (and a
// load's wait lands here, after the independent work placed before it).
template <int N>
__device__ __forceinline__ void pin(float (&x)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) asm volatile("" : "+v"(x[k]));
}
template <int N>
__device__ __forceinline__ void pin_u64(uint64_t (&x)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) asm volatile("" : "+v"(x[k]));
}
__device__ __forceinline__ void pin_u64(uint64_t& x) { asm volatile("" : "+v"(x)); }

// The partial min lives in lane 63 after wave_min63: broadcast it as a wave-uniform value.
__device__ __forceinline__ float uniform_f(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
}

__device__ __forceinline__ float wave_shr1(float x, float old) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                                  __builtin_bit_cast(int, x), 0x138,
                                                                  0xf, 0xf, false));
}


// Every wave publishes, for observation k, two tagged 8-byte words: {partial of k-1, k+1} in
// part[k % kRing][wave] and {boundary of k, k+1} in bnd[k % kRing][wave] (tag 0 = never written).
// Polls read them with relaxed 64-bit atomic loads (ds_read_b64), which the compiler neither
// hoists out of the spin nor merges, and whose lgkmcnt waits it tracks itself.
__device__ __forceinline__ uint64_t lds_load64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint64_t pack(uint32_t tag, float v) {
    return ((uint64_t)tag << 32) | __builtin_bit_cast(uint32_t, v);
}
// The last lane of every row (15, 31, 47, 63; each holds its row's minimum after four DPP
// stages) publishes, with EXEC narrowed inside the asm and restored, so the publish neither
// branches divergently (which would turn the loop counters into VGPRs) nor spends LDS bandwidth
// on idle lanes.  In LDS order (one wave's LDS operations execute in order):
//   ds_write_b32 +inf  -> the cell two observations ahead (wave 0; other waves hit a junk word)
//   ds_min_f32 row min -> this observation's cell
//   ds_add_u32 1       -> this observation's arrival count (a reader that sees every arrival
//                         sees every row's min)
//   ds_write_b64       -> lane 63's tagged last score (lanes 15/31/47: the unused low word)
// Offsets are immediates: the ring slot is a template constant.
template <uint32_t RST_OFF, uint32_t CELL_OFF, uint32_t CNT_OFF, uint32_t BND_OFF>
__device__ __forceinline__ void publish_rows(uint32_t rbase, uint32_t cbase, float rowmin, uint32_t bbase,
                                             uint64_t bndv, float inf, uint32_t one, uint64_t lanes) {
    uint64_t saved;
    asm volatile(
        "s_and_saveexec_b64 %0, %6\n\t"
        "s_nop 1\n\t"
        "ds_write_b32 %1, %7 offset:%9\n\t"
        "ds_min_f32 %2, %3 offset:%10\n\t"
        "ds_add_u32 %2, %8 offset:%11\n\t"
        "ds_write_b64 %4, %5 offset:%12\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "v"(rbase), "v"(cbase), "v"(rowmin), "v"(bbase), "v"(bndv), "s"(lanes), "v"(inf),
          "v"(one), "n"(RST_OFF), "n"(CELL_OFF), "n"(CNT_OFF), "n"(BND_OFF)
        : "memory", "scc");
}

// Row minimum in every lane of a row of 16 (quad swaps, half-row and row mirrors).
__device__ __forceinline__ float row_min16(float x) {
    asm("s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf"
        : "+v"(x));
    return x;
}

// f(integral_constant<int, I>) for I in [I0, N): a loop whose index is a constant expression
template <int I, int N>
struct StaticFor {
    template <class F>
    __device__ __forceinline__ static void run(F& f) {
        f(std::integral_constant<int, I>{});
        StaticFor<I + 1, N>::run(f);
    }
};
template <int N>
struct StaticFor<N, N> {
    template <class F>
    __device__ __forceinline__ static void run(F&) {}
};

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long x;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(x)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return x;
}

// PATHS (decoded paths; HA <= 1, every sequence starts at step 0) adds the backpointers of every
// observation, in the order of the oracle's lexicographic (value, row) argmin.  All of it runs
// after the observation's publish, off the inter-wave critical path:
//   * light position p: its two candidates (position p-1, heavy row 0) are compared in every lane
//     and one bit per lane and slot records "took the heavy term", shifted into a register that
//     holds the last 32 observations and is stored every 32 (PATHS 2: every heavy term wins
//     ties, one compare per slot);
//   * heavy row h: its argmin is re-evaluated by the traceback from the heavy scores and the
//     light minimum of the observation before (wave 0 records them).  Where the light-set term
//     wins or ties, the traceback also needs j* = the lowest light position with
//     fl(c + v[j]) == fl(c + min v): it recomputes that row's light scores from a checkpoint
//     (every kCkptEvery-th row of light scores, stored here) instead of this kernel finding j*
//     for every observation (on 2405.chmm the path needs it about once per sequence).
template <int SM, int W, int HA, bool GE, bool STAMP = false, int DIAG = 0, int PATHS = 0>
__global__ __launch_bounds__(64 * W, (GE && W == 4 && SM <= 10 && HA == 1) ? 4 : 1) void chain_viterbi_kernel(BandModel m, FusedBatch b) {
    static_assert(!PATHS || (HA == 1 && !GE && !STAMP && DIAG == 0), "decoded paths: HA 1, E in VGPRs");
    constexpr int HM = kBandHeavy;
    constexpr uint32_t B = 64 * W;
    extern __shared__ __attribute__((aligned(16))) float lds[];

    const uint32_t n = m.n, erow = m.erow, S = m.S;
    const uint32_t t = threadIdx.x, lane = t & 63u, q = blockIdx.x;
    const uint32_t wave = (uint32_t)uniform((int)(t >> 6));
    if (b.run_mask && b.run_mask[q] == 0) return;  // fallback pass: only the marked rows
    constexpr uint32_t tail = SM * B;
    // diagnostic ablations (never planned): 1 = lane 63 alone publishes, 2 = no arrival check
    // of the partial cells, 4 = no tag check of the boundary words (2 and 4 give wrong results)
    constexpr bool PUB1 = DIAG & 1, NO_MU_WAIT = DIAG & 2, NO_BND_WAIT = DIAG & 4;

    // LDS: heavy constants [kChainMaxSym][kBandTail] | rec [kRing][kMaxWaves][2] (tagged 8 B
    //      words) | cell, count, junk [kRing] | red | symbols [kChainSymChunk] (chain_lds_bytes)
    float* ctab = lds;
    uint64_t* rec = reinterpret_cast<uint64_t*>(lds + kChainMaxSym * kBandTail);
    float* pcell = reinterpret_cast<float*>(rec + 2 * kRing * kMaxWaves);
    uint32_t* pcnt = reinterpret_cast<uint32_t*>(pcell + kRing);
    float* junk = reinterpret_cast<float*>(pcnt + kRing);
    float* red = junk + kRing;
    uint8_t* symr = reinterpret_cast<uint8_t*>(red + 2 * kMaxWaves);  // 16 B aligned

    // ---- resident tables ---------------------------------------------------------------------
    // GE == false: et[s][o] = E[o][position t*SM+s] in VGPRs, picked by s_set_gpr_idx.
    // GE == true:  E rows streamed from L2, [o][t][NQ] float4 per thread, prefetched 4 ahead.
    constexpr int NQ = (SM + 3) / 4;
    f32x32 et[GE ? 1 : SM];
    if constexpr (!GE) {
#pragma unroll
        for (int s = 0; s < SM; ++s)
#pragma unroll
            for (int o = 0; o < kChainMaxSym; ++o)
                et[s][o] = (uint32_t)o < S ? m.erows[(size_t)o * erow + s * B + t] : kInf;
    }
    const float4* __restrict__ er4 = reinterpret_cast<const float4*>(m.erows_t);
    auto load_e4 = [&](uint32_t o, float4 (&d)[NQ]) {
#pragma unroll
        for (int x = 0; x < NQ; ++x) d[x] = er4[((size_t)o * B + t) * NQ + x];
    };
    auto e_from4 = [&](const float4 (&d)[NQ], float (&e)[SM]) {
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            const float4 q4 = d[s / 4];
            e[s] = (s % 4 == 0) ? q4.x : (s % 4 == 1) ? q4.y : (s % 4 == 2) ? q4.z : q4.w;
        }
    };
    // E[o] of the thread's positions
    auto extract = [&](uint32_t o, float (&e)[SM]) {
        if constexpr (GE) {
            float4 d[NQ];
            load_e4(o, d);
            e_from4(d, e);
        } else {
#pragma unroll
            for (int s = 0; s < SM; ++s) e[s] = et[s][o];
            pin(e);  // all SM extractions adjacent: one s_set_gpr_idx_on .. off block
        }
    };
    // Packed fp32: slots (2k, 2k+1) are computed as pairs with v_pk_add_f32 (IEEE adds, bit-identical
    // to two v_add_f32), an odd last slot alone.  The light scores live in pairs
    // P[k] = (slot 2k-1, slot 2k), slot -1 being the chain input p0 of slot 0, so the chain operand
    // of the pair (2k, 2k+1) -- slots (2k-1, 2k) -- is the register pair P[k] itself.
    constexpr int NK = SM / 2, NP = SM / 2 + 1;
    f2 BW2[NK > 0 ? NK : 1], AW2[HA][NK > 0 ? NK : 1];
    float bwS = 0.0f, awS[HA];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        BW2[k] = (f2){m.bw[2 * k * B + t], m.bw[(2 * k + 1) * B + t]};
#pragma unroll
        for (int h = 0; h < HA; ++h)
            AW2[h][k] = (f2){m.aw[(size_t)h * tail + 2 * k * B + t], m.aw[(size_t)h * tail + (2 * k + 1) * B + t]};
    }
    if constexpr (SM & 1) {
        bwS = m.bw[(SM - 1) * B + t];
#pragma unroll
        for (int h = 0; h < HA; ++h) awS[h] = m.aw[(size_t)h * tail + (SM - 1) * B + t];
    }

    for (uint32_t x = t; x < S * kBandTail; x += B)
        ctab[x] = m.erows[(size_t)(x / kBandTail) * erow + tail + x % kBandTail];
    for (uint32_t x = t; x < 2 * kRing * kMaxWaves; x += B) rec[x] = 0ull;  // tag 0: never written
    if (t < kRing) {
        pcell[t] = kInf;
        pcnt[t] = 0;
    }

    // ---- sequence ----------------------------------------------------------------------------
    const uint8_t* sym = b.symbols + b.sym_off[q];
    const uint32_t len = (uint32_t)uniform((int)b.end[q]);
    uint32_t first = (uint32_t)uniform((int)b.begin[q]);
    // symbols [sbase, sbase + kChainSymChunk) staged in LDS (16 B aligned, zero padded source)
    uint32_t sbase = first & ~15u;
    auto stage_symbols = [&]() {
        const uint4* src = reinterpret_cast<const uint4*>(sym + sbase);
        const uint32_t avail = (len + kSymPad - sbase) / 16;
        const uint32_t words = min((uint32_t)kChainSymChunk / 16, avail);
        for (uint32_t x = t; x < words; x += B) reinterpret_cast<uint4*>(symr)[x] = src[x];
    };
    stage_symbols();
    __syncthreads();  // symbols, constants and tags initialised: the only barrier before the epilogue
    f2 P[NP];  // light scores: P[k] = (slot 2k-1, slot 2k) (see the packed-fp32 note above)
    auto vg = [&](int s) -> float { return P[(s + 1) >> 1][(s + 1) & 1]; };
    auto vs = [&](int s, float x) { P[(s + 1) >> 1][(s + 1) & 1] = x; };
    auto vcopy = [&](float (&o)[SM]) {
#pragma unroll
        for (int s = 0; s < SM; ++s) o[s] = vg(s);
    };
    vs(-1, kInf);
    if constexpr (!(SM & 1)) P[NP - 1][1] = kInf;  // unused high half of the last pair
    f2 vh;  // heavy scores (N, C) as one pair: the packed heavy update below and the light rows'
            // broadcast operand (op_sel) read it as a whole
    if (first == 0) {
        const uint32_t o0 = (uint32_t)uniform((int)symr[0]);
        float e0[SM];
        extract(o0, e0);
#pragma unroll
        for (int s = 0; s < SM; ++s) vs(s, e0[s] + m.start[s * B + t]);  // diag(E[s0]) (x) start
#pragma unroll
        for (int h = 0; h < HM; ++h)
            vh[h] = m.hvalid[h] ? ctab[o0 * kBandTail + kBandTailE + h] + m.hstart[h] : kInf;
        first = 1;
    } else {
        const float* vin = b.v_in + (size_t)b.v_in_row[q] * n;
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            const uint32_t r = m.lrow[s * B + t];
            vs(s, r != 0xFFFFFFFFu ? vin[r] : kInf);
        }
#pragma unroll
        for (int h = 0; h < HM; ++h) vh[h] = m.hvalid[h] ? vin[m.hrow[h]] : kInf;
    }

    unsigned long long st_acc[kBandStamps] = {};
    unsigned long long st_prev = 0;
    auto mark = [&](int seg) {
        if constexpr (STAMP) {
            const unsigned long long now = stamp();
            st_acc[seg] += now - st_prev;
            st_prev = now;
        }
    };
    if constexpr (STAMP) st_prev = stamp();

    auto wave_partial = [&](const float* vv) -> float {
        float pm = vv[0];
#pragma unroll
        for (int s = 1; s < SM; ++s) pm = fminf(pm, vv[s]);
        return wave_min63(pm);
    };
    // Exchange per observation k (slot = k % kRing, a template constant in the group loop):
    //   pcell[slot] = min over the rows of every wave (ds_min_f32) -> the min of the light scores
    //                 of k, read by every wave at k+2;
    //   pcnt[slot]  = 4W arrivals per use of the slot (monotonic) say all rows published;
    //   rec[slot][wave].hi = {last score of the wave at k, k+1}, read by wave+1 at k+1.
    // Ring argument (kRing = 8): wave 0 resets cell(k+2) to +inf in its publish of k.  The
    // cell's previous observation k-6 was last read at k-4, and wave 0 publishing k has waited
    // for every wave's publish of k-2 (so they all passed k-4); any wave publishing k+2 has
    // waited for wave 0's publish of k, which LDS executes after the reset.  Tagged records are
    // overwritten two uses after their reader waited on them.  Scores never go denormal (they are
    // sums of -log2 probabilities), so the LDS float min equals fminf up to the sign of zero.
    const uint64_t* const rec_l = rec + 2 * (wave ? wave - 1 : 0) + 1;  // left neighbour (wave 0: itself)
    uint32_t cbase = lds_addr(pcell), rbase = lds_addr(wave ? junk : pcell), one = 1;
    float inf_v = kInf;
    asm volatile("" : "+v"(cbase), "+v"(rbase), "+v"(one), "+v"(inf_v));  // VGPR-resident operands
    const uint32_t bbase = lds_addr(rec + 2 * wave + (lane == 63 ? 1 : 0));
    constexpr uint32_t kCntOff = kRing * 4;
    auto row_partial = [&](const float* vv) -> float {
        float pm = vv[0];
#pragma unroll
        for (int s = 1; s < SM; ++s) pm = fminf(pm, vv[s]);
        if constexpr (PUB1) return wave_min63(pm);  // diagnostic: lane 63 alone publishes
        return row_min16(pm);
    };
    auto publish = [&](auto slotc, uint32_t obs, float rowmin, float vlast) {
        constexpr uint32_t K = decltype(slotc)::value;
        publish_rows<((K + 2) % kRing) * 4, K * 4, kCntOff + K * 4, K * kMaxWaves * 16>(
            rbase, cbase, rowmin, bbase, pack(obs + 1u, vlast), inf_v, one, PUB1 ? 0x8000000000000000ull : 0x8000800080008000ull);
    };
    // Arrivals the count of obs's slot has once every row published obs (obs >= first - 1).
    auto arrivals = [&](uint32_t obs) -> uint32_t { return (PUB1 ? 1u : 4u) * W * (((obs + 1u - first) / kRing) + 1u); };
    // Bounded spins.  `spins` counts slow-path re-reads against kSpinLimit (~0.1 s of s_sleep);
    // past it every wait gives up at once (a broken launch drains) and the epilogue sets the
    // fault word (SVH_E_HIP on the host).  The budget is per symbol chunk, not per sequence: the
    // refill below (every kChainSymChunk = 32768 observations) resets a healthy counter, so a
    // healthy run (well under one re-read per observation) never trips it however long the
    // sequence, while a stuck wait still gives up within one budget.  The reset lives in the
    // refill branch only: per-wait counters or a give-up flag in the wait loops changed the
    // compiler's code for the hot waits and cost 2-14%.  Wave-uniform throughout.
    uint32_t spins = 0, spins_b = 0;  // all slow-path re-reads / those of boundary words
    // min of the light scores of observation obs; (cnt, cell) hold a first read.
    auto take_mu = [&](uint32_t obs, uint32_t slot, uint32_t cnt, float cell) -> float {
        const uint32_t want = arrivals(obs);
        if (!NO_MU_WAIT && __builtin_expect((uint32_t)uniform((int)cnt) < want, 0)) {
            for (uint32_t k = 0;; ++k) {
                if (++spins > kSpinLimit) break;
                if (k >= 2) __builtin_amdgcn_s_sleep(1);  // the first re-reads go straight out
                cnt = __hip_atomic_load(pcnt + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                cell = __hip_atomic_load(pcell + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if ((uint32_t)uniform((int)cnt) >= want) break;
            }
        }
        return cell;
    };
    // the left neighbour's last score of observation obs; `w0` holds a first read of the word
    // (wave 0 reads its own word, which is always current, and takes +inf)
    auto take_bnd = [&](uint32_t obs, uint32_t slot, uint64_t w0) -> float {
        if (W == 1) return kInf;
        uint64_t w = w0;
        if (!NO_BND_WAIT && __builtin_expect(uniform((int)(uint32_t)(w >> 32)) != (int)(obs + 1u), 0)) {
            const uint64_t* bp = rec_l + 2 * kMaxWaves * slot;
            while (true) {
                ++spins_b;
                if (++spins > kSpinLimit) break;
                __builtin_amdgcn_s_sleep(1);
                w = lds_load64(bp);
                if (uniform((int)(uint32_t)(w >> 32)) == (int)(obs + 1u)) break;
            }
        }
        return wave ? __builtin_bit_cast(float, (uint32_t)w) : kInf;
    };
    // heavy constants of symbol o (read one observation before they are needed)
    struct HeavyConst {
        float4 c0;
        float2 c1;
    };
    auto load_heavy = [&](uint32_t o) -> HeavyConst {
        return {*reinterpret_cast<const float4*>(ctab + o * kBandTail),
                *reinterpret_cast<const float2*>(ctab + o * kBandTail + 4)};
    };
    // heavy scores from mu (partials) and their previous values, both rows at once:
    //   vh'[h] = min(fl(A_h + mu), fl(X_hh + vh[h]), fl(X_hk + vh[k]))   (tail: band_tail_x)
    static_assert(kBandTailA == 0 && band_tail_x(0, 0) == 2 && band_tail_x(0, 1) == 4, "tail layout");
    auto heavy_update = [&](float mu, const HeavyConst& hc) {
        const f2 a = (f2){hc.c0.x, hc.c0.y} + (f2){mu, mu};
        const f2 d = (f2){hc.c0.z, hc.c0.w} + vh;
        const f2 x = (f2){hc.c1.x, hc.c1.y} + vh.yx;
        vh = (f2){fminf(fminf(a.x, d.x), x.x), fminf(fminf(a.y, d.y), x.y)};
    };

    // ---- decoded paths ------------------------------------------------------------------------
    // Static lane mask per slot (from pflags): C = the heavy term exists and wins ties (it has the
    // lower row id, or there is no chain term).  The light mask of a slot is [xh < xb] | (C &
    // [xh == xb]): without a heavy term xh = +inf is never below xb and C drops the tie; without
    // a chain term xb = +inf, so the heavy term is taken.
    //
    // Output: the mask words (one per lane and slot) every 32 observations, the checkpoint rows
    // every kCkptEvery, and the heavy records, staged in an LDS ring written by wave 0 (hring
    // [64 rows][kRecWords]) and flushed every 32 observations.
    uint64_t pmC[PATHS ? SM : 1] = {};
    uint32_t macc[PATHS ? SM : 1] = {};  // bit k: record row (last row) - k
    uint32_t* const hring = reinterpret_cast<uint32_t*>(symr + kChainSymChunk);
    uint32_t* const cmq = PATHS ? b.cmask + b.cmask_off[q] : nullptr;
    auto store_masks = [&](uint32_t row0, uint32_t rows) {  // rows row0 .. row0+rows-1, row0 % 32 == 0
#pragma unroll
        for (int s = 0; s < SM; ++s) cmq[((size_t)(row0 >> 5) * SM + s) * B + t] = macc[s] << (32u - rows);
    };
    float* const ckq = PATHS ? b.ckpt + b.ckpt_off[q] : nullptr;
    auto checkpoint = [&](uint32_t obs, const float (&vv)[SM]) {  // obs % kCkptEvery == 0
#pragma unroll
        for (int s = 0; s < SM; ++s) ckq[(size_t)(obs / kCkptEvery) * (SM * B) + s * B + t] = vv[s];
    };
    if constexpr (PATHS) {
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            const uint32_t f = m.pflags[s * B + t];
            const bool ec = f & 1u, ea = f & 2u, hl = f & 4u;
            pmC[s] = __builtin_amdgcn_ballot_w64(ea && (!ec || hl));
        }
        float v0[SM];
        vcopy(v0);
        checkpoint(0, v0);  // v_0
    }
    // Heavy-row record of observation obs (record row obs-1): the inputs of its backpointers --
    // the heavy scores vo of obs-1 and the light minimum mu of obs-1 -- stored by wave 0; the
    // traceback re-evaluates the lexicographic (value, row) argmin from them with the same float
    // operations, only where a path passes.
    auto heavy_record = [&](uint32_t obs, float mu, const float (&vo)[HM]) {
        if (wave == 0 && lane == 0) {
            float* r = reinterpret_cast<float*>(hring + ((obs - 1) & (kPathRing - 1)) * kRecWords);
            r[0] = vo[0];
            r[1] = vo[1];
            r[2] = mu;
        }
    };

    // Flush of the record ring (global layout: kernels.h, FusedBatch::hrec).
    auto flush_recs = [&](uint32_t row0, uint32_t rows) {  // wave 0: rows row0 .. row0+rows-1
        uint32_t* dst = b.hrec + b.hrec_off[q] + (size_t)row0 * kRecWords;
        for (uint32_t x = lane; x < rows * kRecWords; x += 64)
            dst[x] = hring[((row0 + x / kRecWords) & (kPathRing - 1)) * kRecWords + x % kRecWords];
    };
    float own_p1 = kInf, own_p2 = kInf;  // W == 1: partials of the last two observations
    uint32_t pc_next = 0;                 // W > 1: count and cell of the observation before the
    float pm_next = kInf;                 // current one, read half a step before they are needed
    // One observation i with symbol o.  hc_prev: heavy constants of the symbol of i-1.  Order:
    // everything that does not need another wave first; the wave's last score is published before
    // the left neighbour's boundary is consumed (only lane 0's slot 0 needs it), so every exchange
    // has at least one observation of slack.  Returns the heavy constants of o.
    // k3 == i % 4 and lagged == (i > first), both compile-time constants in the group loop.
    auto step = [&](uint32_t i, auto slotc, bool lagged, uint32_t o, const float (&e)[SM],
                    const HeavyConst& hc_prev) -> HeavyConst {
        mark(0);
        constexpr uint32_t s0 = decltype(slotc)::value, s1 = (s0 + kRing - 1) & (kRing - 1),
                           s2 = (s0 + kRing - 2) & (kRing - 1);
        uint32_t pcv = pc_next;  // count and cell of i-2, read during step i-1
        float pmv = pm_next;
        uint64_t bwv = 0;
        if constexpr (W > 1) bwv = lds_load64(rec_l + 2 * kMaxWaves * s1);
        const HeavyConst hc = load_heavy(o);
        // terms that do not need the heavy scores (lane 0's slot 0 is redone below):
        // xb = fl(fl(E + bw) + v_prev), xa = fl(E + aw), in pairs
        vs(-1, wave_shr1(vg(SM - 1), kInf));  // p0
        f2 eb2[NK > 0 ? NK : 1], xb2[NK > 0 ? NK : 1], xa2[HA][NK > 0 ? NK : 1];
        float ebS = 0.0f, xbS = 0.0f, xaS[HA];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const f2 e2 = {e[2 * k], e[2 * k + 1]};
            eb2[k] = e2 + BW2[k];
            xb2[k] = eb2[k] + P[k];
#pragma unroll
            for (int h = 0; h < HA; ++h) xa2[h][k] = e2 + AW2[h][k];
        }
        if constexpr (SM & 1) {
            ebS = e[SM - 1] + bwS;
            xbS = ebS + vg(SM - 2);
#pragma unroll
            for (int h = 0; h < HA; ++h) xaS[h] = e[SM - 1] + awS[h];
        }
        auto xbv = [&](int s) -> float { return (SM & 1) && s == SM - 1 ? xbS : xb2[s >> 1][s & 1]; };
        auto xav = [&](int h, int s) -> float { return (SM & 1) && s == SM - 1 ? xaS[h] : xa2[h][s >> 1][s & 1]; };
        // the exchange reads were issued first; everything above ran while they were in flight
#pragma unroll
        for (int k = 0; k < NK; ++k) asm volatile("" : "+v"(xb2[k]), "+v"(xa2[0][k]));
        if constexpr (SM & 1) asm volatile("" : "+v"(xbS), "+v"(xaS[0]));
        if constexpr (W > 1) {
            if (lagged) asm volatile("" : "+v"(pmv), "+v"(pcv));
        }
        mark(1);
        float mu = kInf, vo[HM];  // PATHS: light minimum and heavy scores of i-2
        if (lagged) {  // heavy scores of i-1
            mu = W > 1 ? take_mu(i - 2, s2, pcv, pmv) : own_p2;
            if constexpr (PATHS) {
#pragma unroll
                for (int h = 0; h < HM; ++h) vo[h] = vh[h];

            }
            heavy_update(mu, hc_prev);
        }
        if constexpr (W > 1) {  // count first, then the cell of i-1 for the next step (LDS keeps the order)
            pc_next = __hip_atomic_load(pcnt + s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            pm_next = __hip_atomic_load(pcell + s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        mark(2);
        float vn[SM];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            f2 r = xb2[k];
#pragma unroll
            for (int h = 0; h < HA; ++h) {
                const f2 x = xa2[h][k] + (f2){vh[h], vh[h]};
                r = (f2){fminf(r.x, x.x), fminf(r.y, x.y)};
            }
            vn[2 * k] = r.x;
            vn[2 * k + 1] = r.y;
        }
        if constexpr (SM & 1) {
            float r = xbS;
#pragma unroll
            for (int h = 0; h < HA; ++h) r = fminf(r, xaS[h] + vh[h]);
            vn[SM - 1] = r;
        }
        mark(3);
        pin(vn);  // the light scores first: the boundary word has had the most time to land
        // lane 0, slot 0: the chain predecessor is the left neighbour's last score of i-1
        float xb0 = 0.0f;
        {
            const float bv = take_bnd(i - 1, s1, bwv);
            float r = (NK > 0 ? eb2[0].x : ebS) + bv;
            if constexpr (PATHS) xb0 = lane == 0 ? r : xbv(0);
#pragma unroll
            for (int h = 0; h < HA; ++h) r = fminf(r, xav(h, 0) + vh[h]);
            vn[0] = lane == 0 ? r : vn[0];
        }
        if constexpr (PATHS) {  // light masks of observation i (record row i-1)
            auto mask_slot = [&](auto sc) {
                constexpr int s = decltype(sc)::value;
                const float xh = xav(0, s) + vh[0];
                const float xbe = s == 0 ? xb0 : xbv(s);
                // heavy term taken: below the chain term, or tied and winning the tie
                if constexpr (PATHS == 2)
                    push_le(macc[s], xh, xbe);
                else
                    push_lt_eqc(macc[s], xh, xbe, pmC[s]);
            };
            StaticFor<0, SM>::run(mask_slot);
        }
        if constexpr (W > 1) {
            publish(slotc, i, row_partial(vn), vn[SM - 1]);
        } else {  // one wave: its own partials are the only ones, keep the last two in registers
            own_p2 = own_p1;
            own_p1 = uniform_f(wave_partial(vn));
        }
        mark(4);
        if constexpr (PATHS) {
            if (lagged) heavy_record(i - 1, mu, vo);  // row i-2
            if constexpr (s0 == 0) {
                if ((i & 31u) == 0) store_masks(i - 32, 32);  // rows i-32 .. i-1 are in macc
                if ((i & (kCkptEvery - 1)) == 0) checkpoint(i, vn);
                if (wave == 0 && (i & 31u) == 8 && i >= 40) flush_recs(i - 40, 32);  // rows complete
            }
        }
#pragma unroll
        for (int s = 0; s < SM; ++s) vs(s, vn[s]);
        return hc;
    };

    // a call with the ring slot of obs as a template constant (head / tail of the loop)
    auto with_slot = [&](uint32_t obs, auto&& fn) {
        switch (obs & (kRing - 1)) {
            case 0: return fn(std::integral_constant<uint32_t, 0>{});
            case 1: return fn(std::integral_constant<uint32_t, 1>{});
            case 2: return fn(std::integral_constant<uint32_t, 2>{});
            case 3: return fn(std::integral_constant<uint32_t, 3>{});
            case 4: return fn(std::integral_constant<uint32_t, 4>{});
            case 5: return fn(std::integral_constant<uint32_t, 5>{});
            case 6: return fn(std::integral_constant<uint32_t, 6>{});
            default: return fn(std::integral_constant<uint32_t, 7>{});
        }
    };
    auto step_rt = [&](uint32_t i, bool lagged, uint32_t o, const float (&e)[SM], const HeavyConst& hcp) -> HeavyConst {
        return with_slot(i, [&](auto kc) { return step(i, kc, lagged, o, e, hcp); });
    };
    if constexpr (W > 1) {
        float v0[SM];
        vcopy(v0);
        const float rm = row_partial(v0);
        with_slot(first - 1, [&](auto kc) { publish(kc, first - 1, rm, v0[SM - 1]); });
    } else {
        float v0[SM];
        vcopy(v0);
        own_p1 = uniform_f(wave_partial(v0));
    }
    auto sym_dword = [&](uint32_t i) -> uint64_t {  // symbols i .. i+7 (i % 8 == 0)
        return *reinterpret_cast<const uint64_t*>(symr + (i - sbase));
    };
    auto sym_of = [](uint64_t w, int k) -> uint32_t { return (uint32_t)uniform((int)((w >> (8 * k)) & 0xFFu)); };
    uint32_t i = first;
    HeavyConst hc = {};
    // head: single steps up to a multiple of 8 (and past `first`, so group steps are lagged)
    for (; i < len && ((i & (kRing - 1)) || i == first); i = (uint32_t)uniform((int)(i + 1))) {
        const uint32_t o = (uint32_t)uniform((int)symr[i - sbase]);
        float e[SM];
        extract(o, e);
        hc = step_rt(i, i > first, o, e, hc);
    }
    // body: groups of eight observations (one ring turn), one symbol dword each; GE: E rows
    // prefetched 4 ahead
    if (i + kRing <= len) {
        uint64_t word = (uint64_t)uniform((int)(uint32_t)sym_dword(i)) |
                        ((uint64_t)(uint32_t)uniform((int)(uint32_t)(sym_dword(i) >> 32)) << 32);
        float4 eb[GE ? 4 : 1][NQ];
        if constexpr (GE) {
#pragma unroll
            for (int k = 0; k < 4; ++k) load_e4(sym_of(word, k), eb[k]);
        }
        for (; i + kRing <= len; i = (uint32_t)uniform((int)(i + kRing))) {
            if (__builtin_expect(i + 2 * kRing > sbase + kChainSymChunk, 0)) {  // uniform: refill (rare)
                __syncthreads();  // every wave is at observation i: the old chunk is dead
                spins = spins > kSpinLimit ? spins : 0u;  // new chunk, new budget (a give-up sticks)
                sbase = i & ~15u;
                stage_symbols();
                __syncthreads();
                const uint64_t w2 = sym_dword(i);
                word = (uint64_t)uniform((int)(uint32_t)w2) | ((uint64_t)(uint32_t)uniform((int)(uint32_t)(w2 >> 32)) << 32);
            }
            const uint64_t next = sym_dword(i + kRing);  // zero padding past len; retired next group
            auto group_step = [&](auto kc) {
                constexpr int k = decltype(kc)::value;
                const uint32_t o = sym_of(word, k);
                float e[SM];
                if constexpr (GE) {
                    e_from4(eb[k & 3], e);
                    // row of observation i+k+4 into the slot just consumed (zero padding: row 0)
                    load_e4(k < 4 ? sym_of(word, k + 4) : sym_of(next, k - 4), eb[k & 3]);
                } else {
                    extract(o, e);
                }
                hc = step(i + k, std::integral_constant<uint32_t, (uint32_t)k>{}, true, o, e, hc);
            };
            group_step(std::integral_constant<int, 0>{});
            group_step(std::integral_constant<int, 1>{});
            group_step(std::integral_constant<int, 2>{});
            group_step(std::integral_constant<int, 3>{});
            group_step(std::integral_constant<int, 4>{});
            group_step(std::integral_constant<int, 5>{});
            group_step(std::integral_constant<int, 6>{});
            group_step(std::integral_constant<int, 7>{});
            word = (uint64_t)uniform((int)(uint32_t)next) | ((uint64_t)(uint32_t)uniform((int)(uint32_t)(next >> 32)) << 32);
        }
    }
    // tail
    for (; i < len; i = (uint32_t)uniform((int)(i + 1))) {
        const uint32_t o = (uint32_t)uniform((int)symr[i - sbase]);
        float e[SM];
        extract(o, e);
        hc = step_rt(i, i > first, o, e, hc);
    }
    if (len > first) {  // heavy scores of the last observation (partials of len-2)
        const uint32_t sl = (len - 2) & (kRing - 1);
        float mu = own_p2;
        if constexpr (W > 1) mu = take_mu(len - 2, sl, pc_next, pm_next);
        if constexpr (PATHS) {  // record row len-2
            float vo[HM];
#pragma unroll
            for (int h = 0; h < HM; ++h) vo[h] = vh[h];
            heavy_update(mu, hc);
            heavy_record(len - 1, mu, vo);
        } else {
            heavy_update(mu, hc);
        }
    }
    if constexpr (PATHS) {
        if (len > 1) {
            // masks not stored by the loop (it stored rows below the last multiple of 32 <= len-1)
            const uint32_t mdone = (len - 1) & ~31u;
            if (mdone < len - 1) store_masks(mdone, len - 1 - mdone);
            if (wave == 0) {
                // records not flushed by the loop (it flushed rows below i-8 at i = 8 mod 32, i >= 40)
                const uint32_t hdone = len - 1 >= 40 ? ((len - 1 - 8) & ~31u) : 0u;
                flush_recs(hdone, len - 1 - hdone);
            }
        }
    }

    if (lane == 0 && m.stamps) {  // diagnostics (SVH_BAND_DEBUG & 4: segment stamps, & 128: spins only)
        mark(5);
        st_acc[6] = spins;
        st_acc[7] = spins_b;
        for (int k = 0; k < kBandStamps; ++k)
            m.stamps[((size_t)q * kMaxWaves + wave) * kBandStamps + k] = st_acc[k];
    }
    if (spins > kSpinLimit && lane == 0 && b.fault) atomicOr(b.fault, kFaultChain);

    // ---- epilogue: scores and the lowest-index argmin ---------------------------------------
    float* out = b.scores + (size_t)q * n;
    float bvv = kInf;
    uint32_t bk = 0xFFFFFFFFu;
#pragma unroll
    for (int s = 0; s < SM; ++s) {
        const uint32_t r = m.lrow[s * B + t];
        if (r != 0xFFFFFFFFu) {
            out[r] = vg(s);
            lex_min(bvv, bk, vg(s), r);
        }
    }
    if (t < (uint32_t)HM && m.hvalid[t]) out[m.hrow[t]] = t ? vh[1] : vh[0];
    if (t == 0) {
#pragma unroll
        for (int h = 0; h < HM; ++h)
            if (m.hvalid[h]) lex_min(bvv, bk, vh[h], (uint32_t)m.hrow[h]);
    }
    wave_lexmin63(bvv, bk);
    uint32_t* redk = reinterpret_cast<uint32_t*>(red + kMaxWaves);
    if (lane == 63) {
        red[wave] = bvv;
        redk[wave] = bk;
    }
    __syncthreads();
    if (t == 0 && b.best) {
        float fv = red[0];
        uint32_t fk = redk[0];
        for (uint32_t w = 1; w < (uint32_t)W; ++w) lex_min(fv, fk, red[w], redk[w]);
        b.best[q] = (fk == 0xFFFFFFFFu) ? -1 : (int64_t)fk;
    }
}

// Instantiated geometries: W waves x SM slots (positions <= 64*W*SM).
template <int W, int HA>
const void* chain_ptr_w(int sm, bool ge) {
    if (ge) {
        switch (sm) {
#define SVH_CASE(SMV) \
    case SMV: return reinterpret_cast<const void*>(&chain_viterbi_kernel<SMV, W, HA, true>);
            SVH_CASE(1) SVH_CASE(2) SVH_CASE(3) SVH_CASE(4) SVH_CASE(5) SVH_CASE(6) SVH_CASE(8)
            SVH_CASE(10) SVH_CASE(12)
#undef SVH_CASE
            default: return nullptr;
        }
    }
    switch (sm) {  // E in VGPRs: <= 5 slots x 32 symbols (6 would spill past 256 VGPRs)
#define SVH_CASE(SMV) \
    case SMV: return reinterpret_cast<const void*>(&chain_viterbi_kernel<SMV, W, HA, false>);
        SVH_CASE(1) SVH_CASE(2) SVH_CASE(3) SVH_CASE(4) SVH_CASE(5)
#undef SVH_CASE
        default: return nullptr;
    }
}

}  // namespace

// Instantiation tables, one translation unit each (they compile in parallel).
const void* chain_fn_ha1(int sm, int waves, bool ge);    // chain_ha1.hip
const void* chain_fn_ha2(int sm, int waves, bool ge);    // chain_ha2.hip
const void* chain_diag_fn(int sm, int waves, bool ge, uint32_t dbg);  // chain_ha1.hip: stamps, ablations
const void* chain_paths_fn(int sm, int waves, bool ties_heavy);  // chain_paths.hip

}  // namespace svh
