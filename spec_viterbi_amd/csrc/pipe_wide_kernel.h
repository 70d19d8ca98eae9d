// Wide pipelined chain Viterbi kernel (gfx950): the throughput plan of the pipelined recurrence
// (pipe.hip, kernels.h PipeModel) for batches that fill the chip.
//
// Reference hot loop: Viterbi_impl/GraphBLAS_impl.cpp:59-73 (same association, bit-identical):
//     v'[j] = min_k fl( fl(E[o][j] + T^T[j][k]) + v[k] )
// Light rows: v'_p = min(fl(eb_p(o) + v_{p-1}), fl(ea_p(o) + F)), eb/ea = fl(E_o[p] + bw/aw) (the
// reference's first add, folded into the table); F speculated as its self loop and checked exactly
// per lane and observation, S as a per-lane recurrence (pipe.hip's header has the argument).
//
// Geometry (the latency plan's transposed): a workgroup owns ONE block of 64*SM positions and
// runs W sequences of it, one per wave.  The block's folded table -- every symbol's (eb, ea) of
// its positions, 8 B per position and symbol -- sits in LDS once and all W waves read it, so the
// table costs LDS bandwidth instead of VGPRs and the per-observation overhead (heavy update,
// boundary exchange, symbol decode) is spread over SM = 8 slots per lane.  Per observation a lane
// reads SM/2 16-byte chunks: [eb_1 .. eb_{SM-1}, eb_0] (slot pairs (1,2), (3,4) ... meet the score
// pairs (v_0,v_1), (v_2,v_3) ... in one v_pk_add_f32 each) and [ea_0 .. ea_{SM-1}] (pairs with
// {F, F}).  Heavy constants come through the scalar cache.
// Block b of sequence q takes its position-0 chain input from block b-1 of q: 8-byte tagged
// granules through L2 as in the latency plan (a 256-observation ring per boundary, prefetched
// four groups of 8 ahead, tag-checked; flow control through the consumer's progress word).
// Workgroups take dynamic tickets (sequence group major, block minor), so a consumer's producer
// has always started: no deadlock beyond residency while nblk workgroups fit on the chip.
// XCD classes (x.xmap, round 6; the latency plan's §5f scheme for a grid of any size): the grid is
// padded to a multiple of 8 nblk and workgroup b takes its ticket from the counter of class
// r = b % 8 (blocks b and b + 8 share an XCD under the observed round-robin placement), whose
// tickets map to a contiguous range of sequence groups, so a group's nblk workgroups share an L2.
// Each workgroup publishes its XCC id; a granule producer whose consumer is on its own XCD stores
// with plain (L2-resident) stores, and so does a consumer with its progress word (SVH_PIPEW_XL);
// otherwise, or when the other's id is not known in time, agent-scope write-through stores.  Per
// class the tickets are still taken in start order, so a consumer's producer has always started.
// Each wave combines its own lanes (S partial, argmin, violation); the last wave of a sequence
// to finish combines the blocks.
//
// Decoded paths (PATHS = 1, 2; pipe_wide_paths.hip): the latency plan's records (pipe_kernel.h)
// in this geometry -- per observation and light position the "took F's term" bit (compare into
// VCC + v_addc into a per-lane word per slot, stored every 32 observations, [word][block][slot]
// [lane]), light-score checkpoints every kCkptEvery observations, F every 32 (block 0) -- and per
// observation ONE heavy partial per block: each lane writes {its light minimum of t-1, its sink
// partial of t} into an LDS ring of 8 rows, and every 8 observations the wave folds the ring
// (lane l reduces row l % 8 over lanes 8(l/8) .. 8(l/8)+7, then across the eight lane groups by
// shuffles) and lanes 0..7 store prec[block][t].  pipe_paths.hip walks the paths from them.
#pragma once
#include "pipe_common.h"

// XCD classes and XCD-local hand-offs for the wide plan (A/B knobs; header comment): the launch's
// row mapping (PipeScratch::xmap, launch_pipew; SVH_PIPEW_XMAP=0 at run time turns it off) and the
// plain stores between workgroups on one XCD.
#ifndef SVH_PIPEW_XL
#define SVH_PIPEW_XL 1
#endif

namespace svh {

using namespace dev;
using namespace pipe_dev;

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// Slot 0's chain term: fl(eb0 + (lane ? x[lane-1] : lane R of bvv)).  DPP reads of bvv and x
// need two wait states after the VALU write of either; the asm provides them (the compiler does
// not see DPP inside asm).  R = 0 takes lane 0 of bvv with a plain add.
template <int R>
__device__ __forceinline__ float chain0(float eb, float bvv, float x) {
    float xb;
    if constexpr (R == 0) {
        asm("v_add_f32_e32 %0, %1, %2\n\t"
            "s_nop 0\n\t"
            "v_add_f32_dpp %0, %3, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb)
            : "v"(bvv), "v"(eb), "v"(x));
    } else {
        asm("s_nop 1\n\t"
            "v_add_f32_dpp %0, %1, %2 row_ror:%4 row_mask:0xf bank_mask:0xf\n\t"
            "v_add_f32_dpp %0, %3, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb)
            : "v"(bvv), "v"(eb), "v"(x), "n"(16 - R));  // lane 0 <- lane R of its row
    }
    return xb;
}

// fl(a + b) per component: one v_pk_add_f32 (measured against two v_add_f32: equal time, fewer
// instructions and registers).
__device__ __forceinline__ f2 pk_add(f2 a, f2 b) { return a + b; }

// Slow-path poll: an agent-scope load that waits for itself, so no load is left pending where
// the slow path rejoins the body (the compiler would otherwise drain every load there).
__device__ __forceinline__ uint64_t g_ld64_sync(const uint64_t* p) {
    uint64_t r;
    asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    return r;
}

template <int SM, int W, bool SX, int PATHS>
__global__ __launch_bounds__(64 * W) void pipew_viterbi_kernel(PipeModel m, FusedBatch b, PipeScratch x,
                                                                const f4* __restrict__ hc4) {
    static_assert(SM % 4 == 0, "slots per lane: a multiple of 4");
    constexpr int NP = SM / 2;                 // slot pairs = 16-byte (eb|ea) chunks per symbol and lane
    constexpr int NC = NP + 1 + (SX ? 1 : 0);  // + heavy constants {A_S A_F X_SS X_FF} [+ {X_SF}]
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t S = m.S, nblk = m.nblk;
    f4* const tabl = reinterpret_cast<f4*>(lds);                        // [S][NC][64]
    float* const ring = lds + (size_t)S * NC * 64 * 4;                  // [W][8][64]
    uint32_t* const tick = reinterpret_cast<uint32_t*>(ring + W * 8 * 64);
    float* const pring = reinterpret_cast<float*>(tick + 4);            // PATHS: [W][8][kPRingStride]

    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t w = (uint32_t)uniform((int)(tid >> 6));
    if (tid == 0) {
        uint32_t t;
        if (x.xmap) {  // class r = b % 8: groups [r gpc, (r + 1) gpc), tickets in start order
            const uint32_t r = blockIdx.x & 7u, gpc = (gridDim.x >> 3) / nblk;
            const uint32_t k = __hip_atomic_fetch_add(x.ctr + kCtrClass + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            t = (r * gpc + k / nblk) * nblk + k % nblk;
        } else {
            t = __hip_atomic_fetch_add(x.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        *tick = t;
    }
    __syncthreads();
    const uint32_t id = (uint32_t)uniform((int)*tick);
    const uint32_t qg = id / nblk, blk = id - qg * nblk;
    {
        // (unrolled: a one-wave workgroup would otherwise wait for each 1 KiB in turn)
        const f4* src = reinterpret_cast<const f4*>(m.tab) + (size_t)blk * S * NC * 64;
#pragma unroll 8
        for (uint32_t i = tid; i < S * NC * 64; i += 64 * W) tabl[i] = src[i];
    }
    __syncthreads();
    const uint32_t ep = (uint32_t)uniform((int)__hip_atomic_load(x.ctr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
    const uint32_t q = qg * W + w;
#if SVH_PIPEW_XL
    const uint32_t my_xcc = xcc_id();
    if (tid == 0 && x.xcc && qg * W < b.nseq)
        __hip_atomic_store(x.xcc + (size_t)qg * nblk + blk, (ep << 4) | my_xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif

    if (q < b.nseq) {
        const uint8_t* __restrict__ sym = b.symbols + b.sym_off[q];
        const uint32_t len = (uint32_t)uniform((int)b.end[q]);
        const uint32_t beg = (uint32_t)uniform((int)b.begin[q]);
        const uint32_t first = beg ? beg : 1u;  // first observation the steps run (state at first-1)
        const int src = blk == 0 ? 0 : 2, dst = blk + 1 < nblk ? 2 : 0;
        const uint32_t p0 = blk * 64 * SM + lane * SM;

        f2 vp[NP];  // light scores of the lane's positions, as pairs (v_0,v_1), (v_2,v_3) ...
        f2 CF;      // {S partial of this lane, F'}
        uint64_t viol = 0;  // lanes where fl(A_F + m) < F' happened (the speculation failed)
        uint32_t spins = 0;
        auto setv = [&](int s, float val) {
            if (s & 1) vp[s >> 1].y = val;
            else vp[s >> 1].x = val;
        };
        if (beg == 0) {
            const uint32_t o0 = (uint32_t)uniform((int)sym[0]);
            const f4 h1 = hc4[o0 * 2 + 1];  // X_SF E_F E_S 0
#pragma unroll
            for (int s = 0; s < SM; ++s) setv(s, m.e0[(size_t)o0 * m.P + p0 + s] + m.start[p0 + s]);
            CF.y = m.rowF >= 0 ? h1.y + m.startF : kInf;
            CF.x = (blk == 0 && lane == 0 && m.rowS >= 0) ? h1.z + m.startS : kInf;
        } else {
            const float* vin = b.v_in + (size_t)b.v_in_row[q] * m.n;
#pragma unroll
            for (int s = 0; s < SM; ++s) {
                const uint32_t r = m.lrow[p0 + s];
                setv(s, r != kNoRow ? vin[r] : kInf);
            }
            CF.y = m.rowF >= 0 ? vin[m.rowF] : kInf;
            CF.x = (blk == 0 && lane == 0 && m.rowS >= 0) ? vin[m.rowS] : kInf;
        }

        // ---- decoded paths (every sequence starts at observation 0): records and tie masks
        // PATHS: the last 32 "took F's term" bits per slot (bit 0 = newest), the static tie masks
        // (PATHS 1), the lane's light minimum of the last step's input scores
        uint32_t macc[PATHS ? SM : 1] = {};
        uint64_t pmC[PATHS ? SM : 1] = {};
        float last_pm = kInf;
        float* const pring_w = pring + w * 8 * kPRingStride;
        uint32_t* const cmq = PATHS ? b.cmask + b.cmask_off[q] : nullptr;
        float* const ckq = PATHS ? b.ckpt + b.ckpt_off[q] : nullptr;
        float2* const precq = PATHS ? b.prec + b.prec_off[q] : nullptr;
        float* const fckq = PATHS ? b.fck + b.fck_off[q] : nullptr;
        const uint32_t wstride = nblk * SM * 64;  // mask words per 32 rows
        auto store_masks = [&](uint32_t word, uint32_t rows) {  // rows 32*word .. +rows-1 are in macc
#pragma unroll
            for (int s = 0; s < SM; ++s)
                cmq[(size_t)word * wstride + (blk * SM + s) * 64 + lane] = macc[s] << (32u - rows);
        };
        auto checkpoint = [&](uint32_t t) {  // t % kCkptEvery == 0: the light scores of t
            f4* d = reinterpret_cast<f4*>(ckq + (size_t)(t / kCkptEvery) * m.P + p0);
#pragma unroll
            for (int c = 0; c < SM / 4; ++c) d[c] = (f4){vp[2 * c].x, vp[2 * c].y, vp[2 * c + 1].x, vp[2 * c + 1].y};
        };
        auto ring_put2 = [&](uint32_t t) {  // {light minimum of t-1, sink partial of t}
            *reinterpret_cast<float2*>(pring_w + (t & 7u) * kPRingStride + lane * 2) = make_float2(last_pm, CF.x);
        };
        // fold rows tb .. tb+7 of the ring (tb % 8 == 0) and store observations t in [1, thi): lane l
        // reduces row l % 8 over lanes 8(l/8) .. +7 (16-byte reads), then over the eight lane groups
        auto fold_ring = [&](uint32_t tb, uint32_t thi) {
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const uint32_t R = lane & 7u, H = lane >> 3;
            const float4* rp = reinterpret_cast<const float4*>(pring_w + R * kPRingStride + H * 16);
            float mm = kInf, cc = kInf;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 e = rp[i];
                mm = fminf(mm, fminf(e.x, e.z));
                cc = fminf(cc, fminf(e.y, e.w));
            }
#pragma unroll
            for (int off = 8; off <= 32; off <<= 1) {
                mm = fminf(mm, __shfl_xor(mm, off));
                cc = fminf(cc, __shfl_xor(cc, off));
            }
            const uint32_t tt = tb + R;
            if (lane < 8 && tt >= 1 && tt < thi) precq[(size_t)blk * len + tt] = make_float2(mm, cc);
        };
        // after the step of observation t (compile-time positions in the unrolled body)
        auto paths_after = [&](uint32_t t, auto maskc, auto ckc, auto foldc) {
            if constexpr (PATHS) {
                ring_put2(t);
                if constexpr (decltype(maskc)::value) {
                    if (t >= 32) store_masks((t >> 5) - 1, 32);
                    if (blk == 0 && lane == 0) fckq[t >> 5] = CF.y;
                }
                if constexpr (decltype(ckc)::value) checkpoint(t);
                if constexpr (decltype(foldc)::value) fold_ring(t - 7, len);
            }
        };
        auto paths_after_rt = [&](uint32_t t) {  // runtime positions (head / tail)
            if constexpr (PATHS) {
                ring_put2(t);
                if ((t & 31u) == 0) {
                    if (t >= 32) store_masks((t >> 5) - 1, 32);
                    if (blk == 0 && lane == 0) fckq[t >> 5] = CF.y;
                }
                if ((t & (kCkptEvery - 1)) == 0) checkpoint(t);
                if ((t & 7u) == 7u) fold_ring(t - 7, len);
            }
        };
        if constexpr (PATHS) {
#pragma unroll
            for (int s = 0; s < SM; ++s) {
                const uint32_t f = m.pflags[p0 + s];
                const bool ec = f & 1u, eaf = f & 2u, hl = f & 4u;
                pmC[s] = __builtin_amdgcn_ballot_w64(eaf && (!ec || hl));
            }
            checkpoint(0);
            if (blk == 0 && lane == 0) fckq[0] = CF.y;
        }

        // ---- symbols: 1024-observation windows in VGPRs (lane l: bytes 16l..16l+15)
        const uint32_t slen = len + kSymPad;
        auto load_window = [&](uint32_t wi) -> uint4 {
            const uint32_t off = wi * kPipeWindow + lane * 16;
            return off < slen ? *reinterpret_cast<const uint4*>(sym + off) : make_uint4(0, 0, 0, 0);
        };
        uint32_t cwi = first >> 10;
        uint4 cw = load_window(cwi), nw = load_window(cwi + 1);
        // The wait budget is per window (as pipe.hip): a new window resets a healthy counter, a
        // give-up sticks.
        auto window_for = [&](uint32_t t) {
            if ((t >> 10) != cwi) {
                cw = nw;
                ++cwi;
                nw = load_window(cwi + 1);
                spins = spins > kSpinLimit ? spins : 0u;
            }
        };
        auto sym1 = [&](uint32_t t) -> uint32_t {
            const uint32_t r = t & 1023u, ln = r >> 4, d = (r >> 2) & 3u;
            const uint32_t wd = d == 0 ? readlane_u(cw.x, ln) : d == 1 ? readlane_u(cw.y, ln)
                              : d == 2 ? readlane_u(cw.z, ln) : readlane_u(cw.w, ln);
            return (wd >> ((r & 3u) * 8)) & 0xFFu;
        };

        // ---- the table chunks of symbol o, heavy constants included (issued one observation
        // before they are used; constants through LDS rather than v_readlane or scalar loads,
        // which would force lgkmcnt(0) and serialise the reads issued a step ahead)
        auto fetch = [&](uint32_t o, f4 (&T)[NC]) {
            const f4* tp = tabl + (size_t)o * (NC * 64) + lane;
#pragma unroll
            for (int c = 0; c < NC; ++c) T[c] = tp[c * 64];
        };
        // ---- one observation with symbol o and its chunks T; bvv lane R = the previous block's
        // last score at t-1
        auto step = [&](uint32_t o, const f4 (&T)[NC], float bvv, auto rc) {
            constexpr int R = decltype(rc)::value;
            auto ebp = [&](int j) -> f2 { return (j & 1) ? T[j >> 1].zw : T[j >> 1].xy; };
            auto eap = [&](int j) -> f2 { return (j & 1) ? T[NP / 2 + (j >> 1)].zw : T[NP / 2 + (j >> 1)].xy; };
            const f2 hs = T[NP].xy, hx = T[NP].zw;  // {A_S, A_F}, {X_SS, X_FF}
            float pm = vp[0].x;  // a serial chain: the compiler folds it into v_min3
#pragma unroll
            for (int s = 1; s < SM; ++s) pm = fminf(pm, (s & 1) ? vp[s >> 1].y : vp[s >> 1].x);
            f2 xb[NP - 1];  // {fl(eb_{2j+1} + v_{2j}), fl(eb_{2j+2} + v_{2j+1})}
#pragma unroll
            for (int j = 0; j < NP - 1; ++j) xb[j] = pk_add(ebp(j), vp[j]);
            const f2 lp = ebp(NP - 1);                                 // {eb_{SM-1}, eb_0}
            const float xbl = lp.x + vp[NP - 1].x;                     // slot SM-1
            const float xb0 = chain0<R>(lp.y, bvv, vp[NP - 1].y);      // slot 0
            const f2 F2 = (f2){CF.y, CF.y};
            f2 xa[NP];
#pragma unroll
            for (int j = 0; j < NP; ++j) xa[j] = pk_add(eap(j), F2);
            // heavy side from the scores of t-1
            const f2 s1 = pk_add(hs, (f2){pm, pm});  // A_S + m, A_F + m
            float xsf = kInf;
            if constexpr (SX) xsf = T[NP + 1].x + CF.y;
            CF = pk_add(hx, CF);                     // X_SS + c, X_FF + F  (F' done)
            {  // viol |= [A_F + m < F'] per lane (an SGPR mask: a per-lane float flag costs registers)
                uint64_t c;
                asm volatile("v_cmp_lt_f32_e64 %1, %2, %3\n\ts_or_b64 %0, %0, %1"
                             : "+s"(viol), "=&s"(c)
                             : "v"(s1.y), "v"(CF.y)
                             : "scc");
            }
            CF.x = fminf(s1.x, CF.x);
            if constexpr (SX) CF.x = fminf(CF.x, xsf);
            // PATHS: F's term taken (row t-1's bit), per slot
            auto push = [&](int s, float a, float bb) {
                if constexpr (PATHS == 2) push_le(macc[s], a, bb);
                else if constexpr (PATHS == 1) push_lt_eqc(macc[s], a, bb, pmC[s]);
            };
            if constexpr (PATHS) {
                last_pm = pm;
                push(0, xa[0].x, xb0);
            }
            vp[0].x = fminf(xa[0].x, xb0);
#pragma unroll
            for (int s = 1; s < SM - 1; ++s) {
                const float b2 = ((s - 1) & 1) ? xb[(s - 1) >> 1].y : xb[(s - 1) >> 1].x;
                const float a2 = (s & 1) ? xa[s >> 1].y : xa[s >> 1].x;
                if constexpr (PATHS) push(s, a2, b2);
                setv(s, fminf(a2, b2));
            }
            if constexpr (PATHS) push(SM - 1, xa[NP - 1].y, xbl);
            vp[NP - 1].y = fminf(xa[NP - 1].y, xbl);
        };

        // ---- exchange state
        float* const ring_w = ring + w * 8 * 64;
        uint64_t* const gin = x.gran + ((size_t)q * (nblk - 1) + (blk - 1)) * kGR;  // src == 2
        uint64_t* const gout = x.gran + ((size_t)q * (nblk - 1) + blk) * kGR;       // dst == 2
        uint64_t* const cons_in = reinterpret_cast<uint64_t*>(x.cons) + (size_t)q * nblk + blk;
        const uint64_t* const cons_out = reinterpret_cast<const uint64_t*>(x.cons) + (size_t)q * nblk + blk + 1;
        float bprev = kInf;  // boundary score of observation t-1 (uniform)

        auto give_up = [&]() -> bool { return ++spins > kSpinLimit; };
        auto gran_value = [&](uint32_t s) -> float {
            const uint64_t* p = gin + (s & (kGR - 1));
            uint64_t gv = g_ld64_sync(p);
            while ((uint32_t)uniform((int)(uint32_t)(gv >> 32)) != gtag(ep, s)) {
                if (give_up()) break;
                __builtin_amdgcn_s_sleep(1);
                gv = g_ld64_sync(p);
            }
            return __builtin_bit_cast(float, (uint32_t)uniform((int)(uint32_t)gv));
        };
        auto cons_ok = [&](uint64_t c, uint32_t need) -> bool {
            return (uint32_t)(c >> 32) == ep && (int)(uint32_t)c >= (int)need;
        };
        auto uni64 = [](uint64_t c) -> uint64_t {
            return (uint64_t)(uint32_t)uniform((int)(uint32_t)c) | ((uint64_t)(uint32_t)uniform((int)(uint32_t)(c >> 32)) << 32);
        };
        auto wait_cons = [&](uint32_t need) {
            uint64_t c = g_ld64_sync(cons_out);
            while (!cons_ok(uni64(c), need)) {
                if (give_up()) break;
                __builtin_amdgcn_s_sleep(2);
                c = g_ld64_sync(cons_out);
            }
        };
        // SVH_PIPEW_XL: is block ob of this group on this wave's XCD?  (a bounded poll of its id; not
        // known in time: no, i.e. write-through stores, always correct)
        auto xcc_local = [&](uint32_t ob) -> bool {
#if SVH_PIPEW_XL
            if (!x.xcc) return false;
            const uint32_t* p = x.xcc + (size_t)qg * nblk + ob;
            for (int i = 0; i < 32; ++i) {
                const uint32_t wv = (uint32_t)uniform((int)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if ((wv >> 4) == (ep & 0x0FFFFFFFu)) return (wv & 0xFu) == my_xcc;
                __builtin_amdgcn_s_sleep(4);
            }
#endif
            (void)ob;
            return false;
        };
        bool gran_plain = false, cons_plain = false;
        // granule / progress-word stores: plain (a relaxed wavefront-scope atomic store: the same
        // unflagged global_store, kept in this XCD's L2) when the reader shares this XCD
        auto st_gran = [&](uint64_t* a, uint64_t v64) {
            if (SVH_PIPEW_XL && gran_plain) __hip_atomic_store(a, v64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            else g_st64(a, v64);
        };
        auto st_cons = [&](uint64_t v64) {
            if (SVH_PIPEW_XL && cons_plain) __hip_atomic_store(cons_in, v64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            else g_st64(cons_in, v64);
        };
        auto put_gran1 = [&](uint32_t s, float val) {
            const uint64_t gv = ((uint64_t)gtag(ep, s) << 32) | __builtin_bit_cast(uint32_t, val);
            if (lane == 0) st_gran(gout + (s & (kGR - 1)), gv);
        };

        auto sweep = [&](auto srcc, auto dstc) {
            constexpr int SRC = decltype(srcc)::value, DST = decltype(dstc)::value;
            using I0 = std::integral_constant<int, 0>;
            if constexpr (SVH_PIPEW_XL && DST == 2) gran_plain = xcc_local(blk + 1);
            if constexpr (SVH_PIPEW_XL && SRC == 2) cons_plain = xcc_local(blk - 1);
            // one observation outside the body (head, tail): per-observation exchange
            auto single = [&](uint32_t t) {
                window_for(t);
                const uint32_t o = (uint32_t)uniform((int)sym1(t));
                if constexpr (DST == 2) {
                    if ((t & 63u) == 0) wait_cons((int)t - (int)kGR + 64);
                }
                f4 T[NC];
                fetch(o, T);
                step(o, T, bprev, I0{});
                paths_after_rt(t);
                if constexpr (DST == 2) {
                    ring_w[(t & 7u) * 64 + lane] = vp[NP - 1].y;  // the body's first store repeats it
                    put_gran1(t, readlane_f(vp[NP - 1].y, 63));
                }
                if constexpr (SRC == 2) {
                    if (t + 1 < len) bprev = gran_value(t);
                    if (lane == 0) st_cons(((uint64_t)ep << 32) | (t + 1));
                }
            };
            // the granules of a group after a tag miss (slow path: poll until the producer has them)
            auto gran_group = [&](uint32_t tg) -> uint64_t {
                uint64_t gv = g_ld64_sync(gin + ((tg + (lane & 7u)) & (kGR - 1)));
                while (__builtin_amdgcn_ballot_w64((uint32_t)(gv >> 32) != gtag(ep, tg)) != 0) {
                    if (give_up()) break;
                    __builtin_amdgcn_s_sleep(1);
                    gv = g_ld64_sync(gin + ((tg + (lane & 7u)) & (kGR - 1)));
                }
                return gv;
            };

            if constexpr (DST == 2) {
                ring_w[((first - 1) & 7u) * 64 + lane] = vp[NP - 1].y;
                put_gran1(first - 1, readlane_f(vp[NP - 1].y, 63));
            }
            if constexpr (SRC == 2) {
                bprev = gran_value(first - 1);
                // initial progress (observations < first are done): a row that starts mid-sequence
                // at a multiple of 64 would otherwise leave its producer's first flow-control wait
                // on a stale word while this wave waits for that producer's granules
                if (lane == 0) st_cons(((uint64_t)ep << 32) | first);
            }

            uint32_t t = first;
            for (; t < len && (t & 31u); ++t) single(t);

            // body: 32 observations per iteration, four groups of 8, in windows of 1024 symbols
            // (one VGPR window load per 32 iterations).  Inside a window every vector-memory
            // operation is unconditional and issued in a fixed order -- per iteration the progress
            // word, per group a granule prefetch (4 groups ahead) and the previous group's granule
            // store, the progress store after group 3 -- and slow paths wait for their own loads,
            // so the compiler's vmcnt before each use counts only younger operations (no drains).
            if (t + 32 <= len) {
                uint64_t cons_v = 0;
                if constexpr (DST == 2) cons_v = g_ld64(cons_out);
                uint64_t gq[4] = {0, 0, 0, 0};  // SRC 2: granule groups in flight
                if constexpr (SRC == 2) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) gq[j] = g_ld64(gin + ((t + 8 * j + (lane & 7u)) & (kGR - 1)));
                }
                // DST 2: the previous group's boundary scores (lanes l: observation gpend_t + l%8),
                // stored one group late; the head's last 8 (or fewer, then slots never read) first
                float gpend = 0.0f;
                if constexpr (DST == 2) gpend = ring_w[(lane & 7u) * 64 + 63];
                uint32_t gpend_t = t - 8;
                auto store_pending = [&]() {
                    st_gran(gout + ((gpend_t + (lane & 7u)) & (kGR - 1)),
                           ((uint64_t)gtag(ep, gpend_t) << 32) | __builtin_bit_cast(uint32_t, gpend));
                };
                float bv_prev = bprev;  // lane 7 (all lanes) = boundary of t-1
                while (t + 32 <= len) {
                  cw = load_window(t >> 10);
                  spins = spins > kSpinLimit ? spins : 0u;  // new window, new budget
                  // wait for the window here (an asm use of it), so no window load is pending at
                  // the inner loop's header (where the compiler would drain every load)
                  asm volatile("" ::"v"(cw.x), "v"(cw.y), "v"(cw.z), "v"(cw.w));
                  const uint32_t wend = ((t >> 10) + 1) << 10;
                  for (; t + 32 <= len && t < wend; t += 32) {
                    const uint32_t r = t & 1023u, ln = r >> 4;
                    const uint64_t sw0 = (uint64_t)readlane_u(cw.x, ln) | ((uint64_t)readlane_u(cw.y, ln) << 32);
                    const uint64_t sw1 = (uint64_t)readlane_u(cw.z, ln) | ((uint64_t)readlane_u(cw.w, ln) << 32);
                    const uint64_t sw2 = (uint64_t)readlane_u(cw.x, ln + 1) | ((uint64_t)readlane_u(cw.y, ln + 1) << 32);
                    const uint64_t sw3 = (uint64_t)readlane_u(cw.z, ln + 1) | ((uint64_t)readlane_u(cw.w, ln + 1) << 32);
                    if constexpr (DST == 2) {  // granule ring flow control, once per 32 observations
                        if (!cons_ok(uni64(cons_v), (int)t + 32 - (int)kGR + 8)) wait_cons((int)t + 32 - (int)kGR + 8);
                    }
                    asm volatile("" ::: "memory");
                    if constexpr (DST == 2) cons_v = g_ld64(cons_out);
                    // chunks of the iteration's first observation; each step fetches the next's
                    f4 Tc[NC];
                    fetch((uint32_t)(sw0 & 0xFFu), Tc);
                    auto group = [&](auto jc, uint64_t sw, uint64_t swn) {
                        constexpr uint32_t j = decltype(jc)::value;
                        const uint32_t tg = t + 8 * j;
                        float bv = kInf;  // lanes 0..7: the previous block's last scores of tg..tg+7
                        if constexpr (SRC == 2) {
                            uint64_t gv = gq[j];
                            if (__builtin_amdgcn_ballot_w64((uint32_t)(gv >> 32) != gtag(ep, tg)) != 0) gv = gran_group(tg);
                            bv = __builtin_bit_cast(float, (uint32_t)gv);
                            asm volatile("" ::: "memory");
                            gq[j] = g_ld64(gin + ((tg + 32 + (lane & 7u)) & (kGR - 1)));
                        }
                        auto one = [&](auto kc) {
                            constexpr uint32_t k = decltype(kc)::value;
                            const uint32_t o = (uint32_t)((sw >> (8 * k)) & 0xFFu);
                            f4 Tn[NC];
                            if constexpr (k < 7) fetch((uint32_t)((sw >> (8 * k + 8)) & 0xFFu), Tn);
                            else if constexpr (j < 3) fetch((uint32_t)(swn & 0xFFu), Tn);
                            // keep the next observation's reads ahead of this step's arithmetic and
                            // the step's arithmetic ahead of the reads after it (the scheduler would
                            // regroup them, and the step's lgkmcnt would then cover the next reads)
                            __builtin_amdgcn_sched_barrier(0);
                            if constexpr (SRC == 0) {
                                step(o, Tc, kInf, I0{});
                            } else if constexpr (k == 0) {
                                step(o, Tc, bv_prev, std::integral_constant<int, 7>{});
                            } else {
                                step(o, Tc, bv, std::integral_constant<int, (int)k - 1>{});
                            }
                            __builtin_amdgcn_sched_barrier(0);
                            if constexpr (k < 7 || j < 3) {
#pragma unroll
                                for (int c = 0; c < NC; ++c) Tc[c] = Tn[c];
                            }
                            if constexpr (DST == 2) ring_w[k * 64 + lane] = vp[NP - 1].y;
                            paths_after(tg + k, std::bool_constant<j == 0 && k == 0>{},
                                        std::bool_constant<k == 0 && (j == 0 || j == 2)>{},
                                        std::bool_constant<k == 7>{});
                        };
                        one(std::integral_constant<uint32_t, 0>{});
                        one(std::integral_constant<uint32_t, 1>{});
                        one(std::integral_constant<uint32_t, 2>{});
                        one(std::integral_constant<uint32_t, 3>{});
                        one(std::integral_constant<uint32_t, 4>{});
                        one(std::integral_constant<uint32_t, 5>{});
                        one(std::integral_constant<uint32_t, 6>{});
                        one(std::integral_constant<uint32_t, 7>{});
                        bv_prev = bv;
                        if constexpr (DST == 2) {
                            asm volatile("" ::: "memory");
                            store_pending();  // all lanes: 8 lanes per granule, same data
                            gpend = ring_w[(lane & 7u) * 64 + 63];
                            gpend_t = tg;
                        }
                        if constexpr (SRC == 2 && j == 3) {
                            asm volatile("" ::: "memory");
                            st_cons(((uint64_t)ep << 32) | (tg + 8));
                        }
                    };
                    group(std::integral_constant<uint32_t, 0>{}, sw0, sw1);
                    group(std::integral_constant<uint32_t, 1>{}, sw1, sw2);
                    group(std::integral_constant<uint32_t, 2>{}, sw2, sw3);
                    group(std::integral_constant<uint32_t, 3>{}, sw3, sw3);
                  }
                }
                bprev = readlane_f(bv_prev, 7);
                if constexpr (DST == 2) store_pending();
                // tail windows
                cwi = t >> 10;
                cw = load_window(cwi);
                nw = load_window(cwi + 1);
            }
            for (; t < len; ++t) single(t);
            if constexpr (PATHS) {
                // rows the loop did not store: masks of rows below len-1 past the last full word,
                // ring rows of the last partial group of 8
                const uint32_t mdone = (len - 1) & ~31u;
                if (mdone < len - 1) store_masks(mdone >> 5, len - 1 - mdone);
                if (((len - 1) & 7u) != 7u) fold_ring((len - 1) & ~7u, len);
            }
        };

        if (len > first && (m.diag & 1u)) {  // diagnostic: no boundary exchange (timing only, wrong results)
            sweep(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
        } else if (len > first) {
            using I0 = std::integral_constant<int, 0>;
            using I2 = std::integral_constant<int, 2>;
            switch (src * 3 + dst) {
                case 0: sweep(I0{}, I0{}); break;
                case 2: sweep(I0{}, I2{}); break;
                case 6: sweep(I2{}, I0{}); break;
                default: sweep(I2{}, I2{}); break;
            }
        }
        if (spins > kSpinLimit && lane == 0 && b.fault) atomicOr(b.fault, kFaultPipeWide);

        // ---- scores of the light positions, this wave's partials, the sequence's combine
        float* out = b.scores + (size_t)q * m.n;
        float bvv = kInf;
        uint32_t bk = kNoRow;
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            const uint32_t r = m.lrow[p0 + s];
            const float val = (s & 1) ? vp[s >> 1].y : vp[s >> 1].x;
            if (r != kNoRow) {
                out[r] = val;
                lex_min(bvv, bk, val, r);
            }
        }
        wave_lexmin63(bvv, bk);
        const float cmin = wave_min63(CF.x);
        if (lane == 63) {
            uint64_t* part = x.part + ((size_t)q * nblk + blk) * 2;
            g_st64(part, ((uint64_t)(viol != 0 ? 1u : 0u) << 32) | __builtin_bit_cast(uint32_t, cmin));
            g_st64(part + 1, lex_key(bvv, bk));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t d = __hip_atomic_fetch_add(x.done + q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (d == nblk - 1) {
                float C = kInf;
                uint64_t key = ~0ull;
                uint32_t vi = 0;
                for (uint32_t u = 0; u < nblk; ++u) {
                    const uint64_t* pu = x.part + ((size_t)q * nblk + u) * 2;
                    const uint64_t a = g_ld64(pu), k2 = g_ld64(pu + 1);
                    C = fminf(C, __builtin_bit_cast(float, (uint32_t)a));
                    vi |= (uint32_t)(a >> 32);
                    key = k2 < key ? k2 : key;
                }
                float bv2 = lex_key_value(key);
                uint32_t bk2 = lex_key_index(key);
                if (key == ~0ull) {
                    bv2 = kInf;
                    bk2 = kNoRow;
                }
                if (m.rowF >= 0) {
                    out[m.rowF] = CF.y;
                    lex_min(bv2, bk2, CF.y, (uint32_t)m.rowF);
                }
                if (m.rowS >= 0) {
                    out[m.rowS] = C;
                    lex_min(bv2, bk2, C, (uint32_t)m.rowS);
                }
                if (b.best) b.best[q] = bk2 == kNoRow ? -1 : (int64_t)bk2;
                x.viol[q] = vi;
                __hip_atomic_store(x.done + q, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    __syncthreads();
    if (tid == 0) {  // launch end: the last workgroup resets the tickets and advances the epoch
        const uint32_t f = __hip_atomic_fetch_add(x.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f == gridDim.x - 1) pipe_reset_counters(x);  // every workgroup has taken its ticket
    }
}

template <int SM, int W, int PATHS>
const void* pipew_ptr(bool sx) {
    return sx ? reinterpret_cast<const void*>(&pipew_viterbi_kernel<SM, W, true, PATHS>)
              : reinterpret_cast<const void*>(&pipew_viterbi_kernel<SM, W, false, PATHS>);
}

}  // namespace

// The kernel's instantiations live in two translation units (they compile in parallel):
// pipe_wide.hip scores (PATHS = 0, 1..16 waves), pipe_wide_paths.hip decoded paths (PATHS 1, 2;
// 1..8 waves: the path ring shares the CU's LDS with the table).  Each returns the kernel for
// (slots, waves, sx, paths) or nullptr.
const void* pipew_kernel_paths(int sm, int waves, bool sx, int paths);

}  // namespace svh
