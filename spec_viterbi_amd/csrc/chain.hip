// Barrier-free chain Viterbi kernel (gfx950) for MSV-shaped models (N, M_1..M_L, C; the shape of
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
#include "device_common.h"
#include "kernels.h"

namespace svh {

using namespace dev;

namespace {

typedef float f32x32 __attribute__((ext_vector_type(32)));

constexpr uint32_t kRing = 4;  // see the ring argument in the step comments
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
// Order-preserving float key (uint order == float order, -0 < +0), and its inverse.
__device__ __forceinline__ uint32_t fkey(float v) {
    const uint32_t b = __builtin_bit_cast(uint32_t, v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float funkey(uint32_t k) {
    return __builtin_bit_cast(float, (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
// Lane 63 alone publishes (EXEC narrowed inside the asm and restored), so the publish neither
// branches divergently (which would turn the loop counters into VGPRs) nor spends LDS bandwidth
// on 63 idle lanes:  ds_max_u64 of {tag, ~key(partial)} into the observation's min cell (larger
// tag wins; within a tag the smallest key), then ds_add_u32 of 1 into its arrival count (LDS
// executes one wave's operations in order, so a reader that sees the count sees the max), then
// the tagged last score.
__device__ __forceinline__ void publish_lane63(uint32_t cell, uint64_t cellv, uint32_t cnt,
                                               uint32_t bnd, uint64_t bndv) {
    uint64_t saved;
    asm volatile(
        "s_and_saveexec_b64 %0, %6\n\t"
        "s_nop 1\n\t"
        "ds_max_u64 %1, %2\n\t"
        "ds_add_u32 %3, %7\n\t"
        "ds_write_b64 %4, %5\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "v"(cell), "v"(cellv), "v"(cnt), "v"(bnd), "v"(bndv), "s"(0x8000000000000000ull), "v"(1u)
        : "memory", "scc");
}

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long x;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(x)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return x;
}

template <int SM, int W, int HA, bool GE, bool STAMP = false>
__global__ __launch_bounds__(64 * W) void chain_viterbi_kernel(BandModel m, FusedBatch b) {
    constexpr int HM = kBandHeavy;
    constexpr uint32_t B = 64 * W;
    extern __shared__ __attribute__((aligned(16))) float lds[];

    const uint32_t n = m.n, erow = m.erow, S = m.S;
    const uint32_t t = threadIdx.x, lane = t & 63u, q = blockIdx.x;
    const uint32_t wave = (uint32_t)uniform((int)(t >> 6));
    constexpr uint32_t tail = SM * B;

    // LDS: heavy constants [kChainMaxSym][kBandTail] | part[kRing][kMaxWaves] | bnd[..] (8 B
    //      tagged words) | red | symbols [kChainSymChunk]
    float* ctab = lds;
    uint64_t* rec = reinterpret_cast<uint64_t*>(lds + kChainMaxSym * kBandTail);  // [kRing][kMaxWaves][2]
    uint64_t* pcell = rec + 2 * kRing * kMaxWaves;                                 // [kRing]
    uint32_t* pcnt = reinterpret_cast<uint32_t*>(pcell + kRing);                   // [kRing] (+pad)
    float* red = reinterpret_cast<float*>(pcnt + 2 * kRing);
    uint8_t* symr = reinterpret_cast<uint8_t*>(red + 2 * kMaxWaves);

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
    float aw[HA][SM], bw[SM];
#pragma unroll
    for (int s = 0; s < SM; ++s) {
        bw[s] = m.bw[s * B + t];
#pragma unroll
        for (int h = 0; h < HA; ++h) aw[h][s] = m.aw[(size_t)h * tail + s * B + t];
    }
    for (uint32_t x = t; x < S * kBandTail; x += B)
        ctab[x] = m.erows[(size_t)(x / kBandTail) * erow + tail + x % kBandTail];
    for (uint32_t x = t; x < 2 * kRing * kMaxWaves + kRing + kRing; x += B) rec[x] = 0ull;  // rec, cells, counts

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
    float v[SM], vh[HM];
    if (first == 0) {
        const uint32_t o0 = (uint32_t)uniform((int)symr[0]);
        float e0[SM];
        extract(o0, e0);
#pragma unroll
        for (int s = 0; s < SM; ++s) v[s] = e0[s] + m.start[s * B + t];  // diag(E[s0]) (x) start
#pragma unroll
        for (int h = 0; h < HM; ++h)
            vh[h] = m.hvalid[h] ? ctab[o0 * kBandTail + kBandTailE + h] + m.hstart[h] : kInf;
        first = 1;
    } else {
        const float* vin = b.v_in + (size_t)b.v_in_row[q] * n;
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            const uint32_t r = m.lrow[s * B + t];
            v[s] = r != 0xFFFFFFFFu ? vin[r] : kInf;
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
    // Exchange per observation k (slot = k % kRing, a compile-time constant in the group loop):
    //   pcell[slot] = max over waves of {k+1, ~key(partial)} -> the min of the light scores of k,
    //   pcnt[slot]  = arrivals (monotonic: W per use of the slot), read by every wave at k+2;
    //   rec[slot][wave].hi = {last score of the wave at k, k+1}, read by wave+1 at k+1.
    const uint64_t* const rec_l = rec + 2 * (wave ? wave - 1 : 0) + 1;  // left neighbour's last scores
    auto publish = [&](uint32_t obs, uint32_t slot, float partial, float vlast) {
        publish_lane63(lds_addr(pcell + slot), ((uint64_t)(obs + 1u) << 32) | (uint64_t)(~fkey(partial)),
                       lds_addr(pcnt + slot), lds_addr(rec + 2 * (slot * kMaxWaves + wave) + 1),
                       pack(obs + 1u, vlast));
    };
    // Arrivals the count of obs's slot has once every wave published obs (obs >= first - 1).
    auto arrivals = [&](uint32_t obs) -> uint32_t { return (uint32_t)W * (((obs + 1u - first) >> 2) + 1u); };
    // Bounded spins: `spins` is wave-uniform (every decision goes through readfirstlane).
    uint32_t spins = 0;
    // min of the light scores of observation obs; (cnt, cell) hold a first read.
    auto take_mu = [&](uint32_t obs, uint32_t slot, uint32_t cnt, uint64_t cell) -> float {
        const uint32_t want = arrivals(obs);
        if (__builtin_expect((uint32_t)uniform((int)cnt) < want, 0)) {
            while (true) {
                if (++spins > kSpinLimit) break;
                __builtin_amdgcn_s_sleep(1);
                cnt = __hip_atomic_load(pcnt + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                cell = lds_load64(pcell + slot);
                if ((uint32_t)uniform((int)cnt) >= want) break;
            }
        }
        return funkey(~(uint32_t)cell);
    };
    // the left neighbour's last score of observation obs; `w0` holds a first read of the word
    auto take_bnd = [&](uint32_t obs, uint32_t slot, uint64_t w0) -> float {
        if (W == 1 || wave == 0) return kInf;
        uint64_t w = w0;
        if (__builtin_expect(uniform((int)(uint32_t)(w >> 32)) != (int)(obs + 1u), 0)) {
            const uint64_t* bp = rec_l + 2 * kMaxWaves * slot;
            while (true) {
                if (++spins > kSpinLimit) break;
                __builtin_amdgcn_s_sleep(1);
                w = lds_load64(bp);
                if (uniform((int)(uint32_t)(w >> 32)) == (int)(obs + 1u)) break;
            }
        }
        return __builtin_bit_cast(float, (uint32_t)w);
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
    // heavy scores from mu (partials) and their previous values
    auto heavy_update = [&](float mu, const HeavyConst& hc) {
        const float cst[6] = {hc.c0.x, hc.c0.y, hc.c0.z, hc.c0.w, hc.c1.x, hc.c1.y};
        float vhn[HM];
#pragma unroll
        for (int h = 0; h < HM; ++h) {
            float a = cst[kBandTailA + h] + mu;
#pragma unroll
            for (int k = 0; k < HM; ++k) a = fminf(a, cst[kBandTailX + h * HM + k] + vh[k]);
            vhn[h] = a;
        }
#pragma unroll
        for (int h = 0; h < HM; ++h) vh[h] = vhn[h];
    };

    float own_p1 = kInf, own_p2 = kInf;  // W == 1: partials of the last two observations
    // One observation i with symbol o.  hc_prev: heavy constants of the symbol of i-1.  Order:
    // everything that does not need another wave first; the wave's last score is published before
    // the left neighbour's boundary is consumed (only lane 0's slot 0 needs it), so every exchange
    // has at least one observation of slack.  Returns the heavy constants of o.
    // k3 == i % 4 and lagged == (i > first), both compile-time constants in the group loop.
    auto step = [&](uint32_t i, uint32_t k3, bool lagged, uint32_t o, const float (&e)[SM],
                    const HeavyConst& hc_prev) -> HeavyConst {
        mark(0);
        const uint32_t s0 = k3 & (kRing - 1), s1 = (k3 + kRing - 1) & (kRing - 1), s2 = (k3 + kRing - 2) & (kRing - 1);
        uint32_t pcv = 0;
        uint64_t pmv = 0;
        if (W > 1 && lagged) {  // count first, then the cell (LDS keeps the order)
            pcv = __hip_atomic_load(pcnt + s2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            pmv = lds_load64(pcell + s2);
        }
        uint64_t bwv = 0;  // wave 0 has no left neighbour: no load (a dead load still costs a wait)
        if (W > 1 && wave) bwv = lds_load64(rec_l + 2 * kMaxWaves * s1);
        const HeavyConst hc = load_heavy(o);
        // terms that do not need the heavy scores (lane 0's slot 0 is redone below)
        const float p0 = wave_shr1(v[SM - 1], kInf);
        float xb[SM], xa[HA][SM];
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            xb[s] = (e[s] + bw[s]) + (s == 0 ? p0 : v[s - 1]);
#pragma unroll
            for (int h = 0; h < HA; ++h) xa[h][s] = e[s] + aw[h][s];
        }
        // the exchange reads were issued first; everything above ran while they were in flight
        pin(xb);
        pin(xa[0]);
        if constexpr (W > 1) {
            if (lagged) {
                pin_u64(pmv);
                asm volatile("" : "+v"(pcv));
            }
            pin_u64(bwv);
        }
        mark(1);
        if (lagged) heavy_update(W > 1 ? take_mu(i - 2, s2, pcv, pmv) : own_p2, hc_prev);  // heavy scores of i-1
        mark(2);
        float vn[SM];
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            float r = xb[s];
#pragma unroll
            for (int h = 0; h < HA; ++h) r = fminf(r, xa[h][s] + vh[h]);
            vn[s] = r;
        }
        mark(3);
        // lane 0, slot 0: the chain predecessor is the left neighbour's last score of i-1
        {
            const float bv = take_bnd(i - 1, s1, bwv);
            float r = (e[0] + bw[0]) + bv;
#pragma unroll
            for (int h = 0; h < HA; ++h) r = fminf(r, xa[h][0] + vh[h]);
            vn[0] = lane == 0 ? r : vn[0];
        }
        const float pi = wave_partial(vn);
        if constexpr (W > 1) {
            publish(i, s0, pi, vn[SM - 1]);
        } else {  // one wave: its own partials are the only ones, keep the last two in registers
            own_p2 = own_p1;
            own_p1 = uniform_f(pi);
        }
        mark(4);
#pragma unroll
        for (int s = 0; s < SM; ++s) v[s] = vn[s];
        return hc;
    };

    if constexpr (W > 1) publish(first - 1, (first - 1) & (kRing - 1), wave_partial(v), v[SM - 1]);
    else own_p1 = uniform_f(wave_partial(v));
    auto sym_word = [&](uint32_t i) -> uint32_t {  // symbols i .. i+3 (i % 4 == 0)
        return *reinterpret_cast<const uint32_t*>(symr + (i - sbase));
    };
    uint32_t i = first;
    HeavyConst hc = {};
    // head: single steps up to a multiple of 4 (and past `first`, so group steps are lagged)
    for (; i < len && ((i & 3u) || i == first); i = (uint32_t)uniform((int)(i + 1))) {
        const uint32_t o = (uint32_t)uniform((int)symr[i - sbase]);
        float e[SM];
        extract(o, e);
        hc = step(i, i & 3u, i > first, o, e, hc);
    }
    // body: groups of four observations, one symbol word each; GE: E rows prefetched 4 ahead
    if (i + 4 <= len) {
        uint32_t word = (uint32_t)uniform((int)sym_word(i));
        float4 eb[GE ? 4 : 1][NQ];
        if constexpr (GE) {
#pragma unroll
            for (int k = 0; k < 4; ++k) load_e4((word >> (8 * k)) & 0xFFu, eb[k]);
        }
        for (; i + 4 <= len; i = (uint32_t)uniform((int)(i + 4))) {
            if (__builtin_expect(i + 8 > sbase + kChainSymChunk, 0)) {  // uniform: refill (rare)
                __syncthreads();  // every wave is at observation i: the old chunk is dead
                sbase = i & ~15u;
                stage_symbols();
                __syncthreads();
                word = (uint32_t)uniform((int)sym_word(i));
            }
            const uint32_t next = sym_word(i + 4);  // zero padding past len; retired next group
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t o = (uint32_t)uniform((int)((word >> (8 * k)) & 0xFFu));
                float e[SM];
                if constexpr (GE) {
                    e_from4(eb[k], e);
                    // row of observation i+k+4 into the slot just consumed (zero padding: row 0)
                    load_e4((uint32_t)uniform((int)((next >> (8 * k)) & 0xFFu)), eb[k]);
                } else {
                    extract(o, e);
                }
                hc = step(i + k, (uint32_t)k, true, o, e, hc);
            }
            word = (uint32_t)uniform((int)next);
        }
    }
    // tail
    for (; i < len; i = (uint32_t)uniform((int)(i + 1))) {
        const uint32_t o = (uint32_t)uniform((int)symr[i - sbase]);
        float e[SM];
        extract(o, e);
        hc = step(i, i & 3u, i > first, o, e, hc);
    }
    if (len > first) {  // heavy scores of the last observation (partials of len-2)
        const uint32_t sl = (len - 2) & (kRing - 1);
        float mu = own_p2;
        if constexpr (W > 1) {
            const uint32_t c = __hip_atomic_load(pcnt + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            mu = take_mu(len - 2, sl, c, lds_load64(pcell + sl));
        }
        heavy_update(mu, hc);
    }

    if constexpr (STAMP) {
        if (lane == 0 && m.stamps) {
            mark(5);
            st_acc[6] = spins;
            for (int k = 0; k < kBandStamps; ++k)
                m.stamps[((size_t)q * kMaxWaves + wave) * kBandStamps + k] = st_acc[k];
        }
    }
    if (spins > kSpinLimit && lane == 0 && m.fault) atomicOr(m.fault, 1u);

    // ---- epilogue: scores and the lowest-index argmin ---------------------------------------
    float* out = b.scores + (size_t)q * n;
    float bvv = kInf;
    uint32_t bk = 0xFFFFFFFFu;
#pragma unroll
    for (int s = 0; s < SM; ++s) {
        const uint32_t r = m.lrow[s * B + t];
        if (r != 0xFFFFFFFFu) {
            out[r] = v[s];
            lex_min(bvv, bk, v[s], r);
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
const void* chain_fn(int sm, int waves, int ha, bool ge) {
    return ha == 1 ? chain_ptr<1>(sm, waves, ge) : ha == 2 ? chain_ptr<2>(sm, waves, ge) : nullptr;
}

}  // namespace

bool chain_supported(int sm, int waves, int ha, bool ge) { return chain_fn(sm, waves, ha, ge) != nullptr; }

hipError_t launch_chain(const BandModel& m, int ha, const FusedBatch& b, hipStream_t stream) {
    const int waves = (int)(m.B / 64);
    const bool ge = m.ge != 0;
    const void* fn = chain_fn((int)m.SM, waves, ha, ge);
    if ((m.dbg & 4u) && ha == 1) {  // diagnostic stamp builds
        if (!ge && m.SM == 5 && waves == 8) fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<5, 8, 1, false, true>);
        if (!ge && m.SM == 5 && waves == 1) fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<5, 1, 1, false, true>);
        if (ge && m.SM == 10 && waves == 4) fn = reinterpret_cast<const void*>(&chain_viterbi_kernel<10, 4, 1, true, true>);
    }
    if (!fn || m.B % 64 || m.S > (uint32_t)kChainMaxSym || m.erow < m.SM * m.B + kBandTail ||
        (ge && !m.erows_t))
        return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    BandModel mm = m;
    FusedBatch bb = b;
    void* args[] = {&mm, &bb};
    return hipLaunchKernel(fn, dim3(b.nseq), dim3(m.B), args, chain_lds_bytes(), stream);
}

}  // namespace svh
