// Diagonal plan of the chain Viterbi step (gfx950): the scores path of MSV-shaped models
// (kernels.h, PipeModel) for batches up to a few hundred sequences.
//
// Reference hot loop: Viterbi_impl/GraphBLAS_impl.cpp:59-73 (same association, bit-identical):
//     v'[j] = min_k fl( fl(E[o][j] + T^T[j][k]) + v[k] )
// For the light rows of the chain shape, with F's light term speculated away as in pipe_kernel.h
// (F'(t) = fl(X_FF(o_t) + F'(t-1)), checked exactly at every observation),
//     v_p(t) = min( fl(eb_p(o_t) + v_{p-1}(t-1)), fl(ea_p(o_t) + F'(t-1)) )
// depends on ONE score of the previous observation: position p-1's.  The pipelined plan
// (pipe_kernel.h) gives a wave a block of positions and hands the block's last score to the next
// wave every observation -- a chain of 19 waves whose exchange and fill cost a third of its time
// (DESIGN.md 5k).  Here a lane follows an anti-diagonal instead: lane l of range r holds, after
// step i, position p = (64 r + l + i) mod NP (NP = 64 x ranges >= light rows; positions past the
// last light row are +inf dummies), so the score it needs, v_{p-1}(t-1), is its own previous value.
// No lane ever reads another lane's score: no exchange, no fill, no inter-wave wait.
// Position 0 has no chain term (eb_0 = +inf), so a lane wrapping from NP-1 to 0 starts a fresh
// diagonal from F' alone, exactly as the recurrence does.
//
// What each step needs besides the lane's own score:
//   * the table pair {ea_p(o_t), eb_p(o_t)} of the lane's position: a ring in LDS holds the last
//     160 table columns the workgroup's lanes walk through, for every symbol ([S][kDR + 64 mirror]
//     float2, so the 64 lanes' read is one contiguous ds_read_b64 at any ring offset); five groups of
//     32 columns, one refilled per block of 32 steps, two groups ahead of use (global loads one block
//     before their LDS writes; one s_barrier per block), so a block's last steps can read the next
//     block's first pairs ahead of time;
//   * the uniform constants of o_t: a per-wave stream in LDS, one 32-byte entry per step
//     {A_F, A_S, X_FF, X_SF, X_SS, ring address of (o_t, step)}, built one block ahead from the
//     sequence's symbols (two broadcast reads per step).
// The steps are software-pipelined: a stream entry is read kPS steps and a ring pair kPE steps
// before its use (the ring address comes from the stream), across block boundaries too.
// A workgroup is W sequences x one range of 64 diagonals: its waves walk the same ring columns
// (shared ring), each with its own sequence's symbols.
// Per step and lane (wave64):  Y = {x, x} + {A_F, A_S};  W = {F, F} + {X_FF, X_SF};
//   Z = {ea, eb} + {F, x};  x' = min(Z.eb, Z.ea);  c' = min(fl(X_SS + c), Y.A_S, W.X_SF);
//   viol += [Y.A_F < W.X_FF];  F' = W.X_FF
// -- three v_pk_add_f32, five VALU more, three LDS reads.  The sink S and the violation check
// are lane-local exactly as in pipe_kernel.h (S(t) = min over lanes of a per-lane recurrence driven
// by the lane's own scores: fl(a + .) is monotone; the lane holding the S(0) chain is range 0's
// lane 0).  F' is computed by every wave redundantly (the same operations: bit-identical).
// The last wave of a sequence to finish combines the ranges' partials (S, argmin, violation); a
// row whose check failed is re-run exactly by that wave's workgroup (pipe_rerun_row) in the same
// launch.
#include "pipe_kernel.h"

#include <cstdlib>

namespace svh {

namespace {

#ifndef SVH_DIAG_K
#define SVH_DIAG_K 64
#endif
constexpr uint32_t kDK = SVH_DIAG_K;  // steps per block (= columns per ring group; 32 or 64)
static_assert(kDK == 32 || kDK == 64, "block length");
constexpr uint32_t kDR = 5 * kDK;     // ring columns (five groups of kDK)
constexpr uint32_t kDRS = kDR + 64;   // slots per symbol plane: the ring and a mirror of its first 64
constexpr uint32_t kDG = kDR / kDK;   // ring groups
constexpr uint32_t kCP = kDK / 2;     // 16-byte chunks of a plane's group (two columns each)
constexpr uint32_t kDE = 8;           // floats per stream entry
#ifndef SVH_DIAG_PS
#define SVH_DIAG_PS 6
#endif
#ifndef SVH_DIAG_PE
#define SVH_DIAG_PE 2
#endif
constexpr uint32_t kPS = SVH_DIAG_PS;  // steps a stream entry is read ahead of its use (two at a time)
constexpr uint32_t kPE = SVH_DIAG_PE;  // steps a ring pair is read ahead of its use (< kPS)
constexpr uint32_t kNS = kPS + 2;      // stream registers: entries j .. j + kPS - 1 and the two being read
static_assert(kPE < kPS && kPS % 2 == 0 && kDK % kNS == 0 && kDK % kPE == 0,
              "prefetch distances: the register slots of step j (j % kNS, j % kPE) repeat every block");
constexpr uint32_t kDMaxSym = 32;
// SVH_DIAG_AB (diagnostic builds, timing only, wrong results): 1 = no stream reads in the steps
// (every step takes the block's first entry), 2 = no ring reads (the prologue's pairs), 3 = no
// barrier between blocks, 4 = no prologue table loads, 5 = no partials / combine, 6 = return at entry,
// 7 = no arrival count (the last range combines), 8 = the arrival count without the combine
#ifndef SVH_DIAG_AB
#define SVH_DIAG_AB 0
#endif
#ifndef SVH_DIAG_FINISH
#define SVH_DIAG_FINISH 0
#endif
#ifndef SVH_DIAG_DONE_STRIDE  // words between rows' arrival counts (the scratch holds 32 per row)
#define SVH_DIAG_DONE_STRIDE 1
#endif

__device__ __forceinline__ f2 lds_ld2(uint32_t a) {
    return *(const __attribute__((address_space(3))) f2*)(size_t)a;
}

// viol += [a < b]: the compare into VCC and v_addc with VCC as the carry-in (two VALU; the compiler's
// compare / v_cndmask / add needs a wait state besides)
__device__ __forceinline__ void push_lt(uint32_t& acc, float a, float b) {
    asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n\t"
                 "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc"
                 : "+v"(acc)
                 : "v"(a), "v"(b)
                 : "vcc");
}

__host__ __device__ constexpr size_t diag_lds_main(uint32_t W, uint32_t S) {
    // ring [S][kDRS] float2 | symbol template [S][8] | streams [W][2][kDK][kDE] | blocks [W] | rerun rows [W]
    return ((size_t)S * kDRS * 2 + (size_t)S * 8 + (size_t)W * 2 * kDK * kDE + 2 * W) * 4;
}

template <int W, bool SX>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(2)))
void diag_viterbi_kernel(PipeModel m, FusedBatch b, PipeScratch x) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t S = m.S, NR = m.nrng, NP = NR * 64, P = m.P;
    float* ring = lds;                                   // [S][kDRS] {ea, eb}
    float* hcr = ring + (size_t)S * kDRS * 2;            // [S][8] stream template of symbol o
    float* strm = hcr + S * 8;                           // [W][2][kDK][kDE]
    uint32_t* wnb = reinterpret_cast<uint32_t*>(strm + W * 2 * kDK * kDE);  // [W] blocks of wave w
    uint32_t* rrow = wnb + W;                            // [W] row wave w's combine hands to the re-run

    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t w = (uint32_t)uniform((int)(tid >> 6));
    const uint32_t rg = blockIdx.x % NR, grp = blockIdx.x / NR;
    const uint32_t q = grp * W + w;
    const bool real = q < b.nseq;
    const uint32_t ring_a = lds_addr(ring);

    // stream template: {A_F, A_S, X_FF, X_SS, X_SF, LDS address of plane o, 0, 0}
    for (uint32_t i = tid; i < S * 8; i += 64 * W) {
        const uint32_t o = i >> 3, k = i & 7u;
        const float* h = m.hc + o * 8;  // A_S A_F X_SS X_FF | X_SF E_F E_S 0
        float v = 0.0f;
        if (k == 0) v = h[1];
        else if (k == 1) v = h[0];
        else if (k == 2) v = h[3];
        else if (k == 3) v = h[2];
        else if (k == 4) v = SX ? h[4] : kInf;
        else if (k == 5) v = __builtin_bit_cast(float, ring_a + o * kDRS * 8u);
        hcr[i] = v;
    }

    const uint8_t* __restrict__ sym = b.symbols + (real ? b.sym_off[q] : 0);
    const uint32_t len = real ? (uint32_t)uniform((int)b.end[q]) : 0u;
    const uint32_t beg = real ? (uint32_t)uniform((int)b.begin[q]) : 0u;
    const uint32_t first = beg ? beg : 1u;                // first observation the steps run (state at first-1)
    const uint32_t nst = len > first ? len - first : 0u;  // steps: observations first .. len-1
    const uint32_t nb = (nst + kDK - 1) / kDK;
    if (lane == 0) {
        wnb[w] = nb;
        rrow[w] = kNoRow;
    }

    // ---- ring refill: group g = columns u in [kDK g, kDK g + kDK) of this range (table column
    // (64 rg + u) mod NP), every symbol plane; 16 chunks of 16 bytes per plane over the workgroup
    constexpr uint32_t kT = 64 * W;
    constexpr uint32_t kRep = (kCP * kDMaxSym + kT - 1) / kT;
    const uint32_t nchunk = kCP * S;
    typedef float lvec __attribute__((ext_vector_type(4 * kRep)));  // a vector, not an array: stays in VGPRs
    lvec lreg;
    auto gload = [&](uint32_t g) {
        const uint32_t c0 = (rg * 64 + g * kDK) % NP;
#pragma unroll
        for (uint32_t r = 0; r < kRep; ++r) {
            // unconditional (clamped) loads: the registers stay registers
            const uint32_t k = min(tid + r * kT, nchunk - 1);
            const float4 v = *reinterpret_cast<const float4*>(m.dtab + (size_t)(k / kCP) * NP + c0 + 2 * (k % kCP));
            lreg[4 * r] = v.x;
            lreg[4 * r + 1] = v.y;
            lreg[4 * r + 2] = v.z;
            lreg[4 * r + 3] = v.w;
        }
    };
    auto lwrite = [&](uint32_t g) {
        const uint32_t s0 = (g % kDG) * kDK;
#pragma unroll
        for (uint32_t r = 0; r < kRep; ++r) {
            const uint32_t k = tid + r * kT;
            if (k < nchunk) {
                float* d = ring + ((size_t)(k / kCP) * kDRS + s0 + 2 * (k % kCP)) * 2;
                const float4 v = make_float4(lreg[4 * r], lreg[4 * r + 1], lreg[4 * r + 2], lreg[4 * r + 3]);
                *reinterpret_cast<float4*>(d) = v;
                if (s0 < 64) *reinterpret_cast<float4*>(d + kDR * 2) = v;
            }
        }
    };
    // ---- per-wave stream of block kb (steps kDK kb + 1 + j, step i reading observation first - 1 + i):
    // lane j builds entry j from the symbol it loaded one block earlier
    uint32_t symv = 0;
    auto symload = [&](uint32_t kb) {
        const uint32_t t = first + kb * kDK + lane;
        const uint32_t tc = t < len ? t : (len ? len - 1 : 0u);
        symv = (real && lane < kDK) ? (uint32_t)sym[tc] : 0u;
    };
    auto sbuild = [&](uint32_t kb) {
        if (lane < kDK) {
            const uint32_t o = symv < S ? symv : 0u;
            const float4 h0 = *reinterpret_cast<const float4*>(hcr + o * 8);
            float4 h1 = *reinterpret_cast<const float4*>(hcr + o * 8 + 4);
            const uint32_t i = kb * kDK + 1 + lane;
            h1.y = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, h1.y) + (i % kDR) * 8u);
            float* d = strm + ((w * 2 + (kb & 1u)) * kDK + lane) * kDE;
            *reinterpret_cast<float4*>(d) = h0;
            *reinterpret_cast<float4*>(d + 4) = h1;
        }
    };

    // ---- prologue: groups 0..3 in the ring, group 4 in flight; the stream of block 0
#if SVH_DIAG_AB == 6  // diagnostics: the launch alone
    return;
#endif
#if SVH_DIAG_AB != 4  // diagnostics: no prologue table loads (rows of one observation stay exact)
    gload(0);
    lwrite(0);
    gload(1);
    lwrite(1);
    gload(2);
    lwrite(2);
    gload(3);
    lwrite(3);
    gload(4);
#endif
    symload(0);
    __syncthreads();  // the symbol template
    sbuild(0);
    symload(1);

    // ---- state at observation first - 1
    float xv = kInf, F = kInf, c = kInf;
    uint32_t viol = 0;
    if (real && beg == 0) {
        const uint32_t o0 = (uint32_t)uniform((int)sym[0]);
        const uint32_t p = rg * 64 + lane;
        xv = m.e0[(size_t)o0 * P + p] + m.start[p];
        F = m.rowF >= 0 ? m.hc[o0 * 8 + 5] + m.startF : kInf;
        c = (rg == 0 && lane == 0 && m.rowS >= 0) ? m.hc[o0 * 8 + 6] + m.startS : kInf;
    } else if (real) {  // resumed row (the _spec tail, time-parallel segments): scores of first-1
        const float* vin = b.v_in + (size_t)b.v_in_row[q] * m.n;
        const uint32_t r = m.lrow[rg * 64 + lane];
        xv = r != kNoRow ? vin[r] : kInf;
        F = m.rowF >= 0 ? vin[m.rowF] : kInf;
        c = (rg == 0 && lane == 0 && m.rowS >= 0) ? vin[m.rowS] : kInf;
    }
    __syncthreads();  // ring groups 0..3, wnb
    uint32_t nbmax = 0;
#pragma unroll
    for (int u = 0; u < W; ++u) nbmax = wnb[u] > nbmax ? wnb[u] : nbmax;
    nbmax = (uint32_t)uniform((int)nbmax);

    // software pipeline: stream entries of steps j .. j + kPS + 1 and ring pairs of j .. j + kPE - 1
    // in registers (slot j % kNS, j % kPE)
    typedef float hvec __attribute__((ext_vector_type(4 * kNS)));
    typedef float gvec __attribute__((ext_vector_type(2 * kNS)));
    typedef float evec __attribute__((ext_vector_type(2 * kPE)));
    hvec hq;
    gvec gq;
    evec eq;
    auto sread = [&](uint32_t kb, uint32_t j, uint32_t slot) {  // stream entry j of block kb (j < 2 kDK)
        const float* st = strm + ((w * 2 + ((kb + j / kDK) & 1u)) * kDK + j % kDK) * kDE;
        const float4 h = *reinterpret_cast<const float4*>(st);
        const float2 g = *reinterpret_cast<const float2*>(st + 4);
        hq[4 * slot] = h.x;
        hq[4 * slot + 1] = h.y;
        hq[4 * slot + 2] = h.z;
        hq[4 * slot + 3] = h.w;
        gq[2 * slot] = g.x;
        gq[2 * slot + 1] = g.y;
    };
    auto eread = [&](uint32_t sslot, uint32_t eslot) {
        // (the element copied to a scalar first: __builtin_bit_cast of an ext-vector element lvalue
        // reads the vector's first element)
        const float roff = gq[2 * sslot + 1];
        const f2 e = lds_ld2(__builtin_bit_cast(uint32_t, roff) + lane * 8u);
        eq[2 * eslot] = e.x;
        eq[2 * eslot + 1] = e.y;
    };
#pragma unroll
    for (uint32_t j = 0; j < kPS; ++j) sread(0, j, j);
#pragma unroll
    for (uint32_t j = 0; j < kPE; ++j) eread(j, j);

    // the state as two register pairs: {F, c} (the feeder and the lane's sink partial: one packed add
    // advances both, {X_FF + F, X_SS + c}) and {x, -} (the lane's score: the source of the packed
    // heavy terms {A_F + x, A_S + x})
    f2 FC = (f2){F, c};
    f2 XP = (f2){xv, 0.0f};
    auto step = [&](const float4& h, const float2& g2, const f2& e) {
        const f2 Y = XP.xx + (f2){h.x, h.y};  // {A_F + x, A_S + x}
        const f2 Wv = FC + (f2){h.z, h.w};    // {F' = X_FF + F, X_SS + c}
        const float za = e.x + FC.x;          // ea + F
        const float zb = e.y + XP.x;          // eb + x
        float cn = fminf(Wv.y, Y.y);
        if (SX) cn = fminf(cn, g2.x + FC.x);  // X_SF + F
        push_lt(viol, Y.x, Wv.x);             // the speculation check: F' would have taken A_F + x
        XP.x = fminf(zb, za);
        FC = (f2){Wv.x, cn};
    };
    auto blockwork = [&](uint32_t kb) {
        lwrite(kb + 4);  // into the slots of group kb - 1, which no wave reads any more
        gload(kb + 5);
        sbuild(kb + 1);  // into the buffer of block kb - 1 (the last steps of block kb read its first entries)
        symload(kb + 2);
    };
    auto block = [&](uint32_t kb) {
#pragma unroll
        for (uint32_t j = 0; j < kDK; ++j) {
            const uint32_t a = SVH_DIAG_AB == 1 ? 0u : j % kNS, b2 = j % kPE;
            const float4 h = make_float4(hq[4 * a], hq[4 * a + 1], hq[4 * a + 2], hq[4 * a + 3]);
            const float2 g2 = make_float2(gq[2 * a], gq[2 * a + 1]);
            const f2 e = (f2){eq[2 * b2], eq[2 * b2 + 1]};
            if (SVH_DIAG_AB != 2) eread((j + kPE) % kNS, j % kPE);  // ring pair of step j + kPE
            // stream entries of steps j + kPS and j + kPS + 1 (the next block's past 31), read together
            // at even steps (the two address words go out as one ds_read2_b32)
            if (SVH_DIAG_AB != 1 && j % 2 == 0) {
                sread(kb, j + kPS, (j + kPS) % kNS);
                sread(kb, j + kPS + 1, (j + kPS + 1) % kNS);
            }
            step(h, g2, e);
            if (j % 2 == 1) __builtin_amdgcn_sched_barrier(0);  // keep the reads where they are issued
        }
    };
    // the row's last, partial block: plain steps
    auto tail = [&](uint32_t kb, uint32_t rem) {
        const float* st = strm + (w * 2 + (kb & 1u)) * kDK * kDE;
        for (uint32_t j = 0; j < rem; ++j) {
            const float4 h = *reinterpret_cast<const float4*>(st + j * kDE);
            const float2 g2 = *reinterpret_cast<const float2*>(st + j * kDE + 4);
            step(h, g2, lds_ld2(__builtin_bit_cast(uint32_t, g2.y) + lane * 8u));
        }
    };

    for (uint32_t k = 0; k < nbmax; ++k) {
        const uint32_t rem = k < nb ? nst - k * kDK : 0u;
        const bool full = k < nb && rem >= kDK;
        // (issuing this work between the block's steps instead measured the same: 0.1940 against
        // 0.1934 ms; the per-block cost is the barrier and its LDS drain, profiles/r06_diag/)
        blockwork(k);
        if (k < nb) {
#ifdef SVH_DIAG_SIMPLE  // diagnostics: every block through the plain steps (no software pipeline)
            tail(k, rem >= kDK ? kDK : rem);
#else
            if (full) block(k);
            else tail(k, rem);
#endif
        }
        if (SVH_DIAG_AB != 3) lds_barrier();
    }

    F = FC.x;
    c = FC.y;
    xv = XP.x;

    // ---- scores of the light positions and this wave's partials
#if SVH_DIAG_AB == 5  // diagnostics: the scores only (every wave leaves here)
    if (real && m.lrow[(rg * 64 + lane + nst) % NP] != kNoRow)
        g_st_score(b.scores + (size_t)q * m.n + m.lrow[(rg * 64 + lane + nst) % NP], xv);
    return;
#endif
#if SVH_DIAG_FINISH  // partials only: diag_finish_kernel combines them after this launch
    if (real) {
        float* out = b.scores + (size_t)q * m.n;
        const uint32_t r = m.lrow[(rg * 64 + lane + nst) % NP];
        float bv = kInf;
        uint32_t bk = kNoRow;
        if (r != kNoRow) {
            out[r] = xv;
            bv = xv;
            bk = r;
        }
        wave_lexmin63(bv, bk);
        const float cmin = wave_min63(c);
        const bool any_viol = __builtin_amdgcn_ballot_w64(viol != 0) != 0;
        if (lane == 63) {
            uint64_t* part = x.part + ((size_t)q * x.G + rg) * 2;
            part[0] = ((uint64_t)(any_viol ? 1u : 0u) << 32) | __builtin_bit_cast(uint32_t, cmin);
            part[1] = lex_key(bv, bk);
            if (rg == 0 && m.rowF >= 0) out[m.rowF] = F;
        }
    }
    return;
#endif
    uint32_t last = 0;
    if (real) {
        float* out = b.scores + (size_t)q * m.n;
        const uint32_t pe = (rg * 64 + lane + nst) % NP;
        const uint32_t r = m.lrow[pe];
        float bv = kInf;
        uint32_t bk = kNoRow;
        if (r != kNoRow) {
            g_st_score(out + r, xv);  // the row's re-run may come from another XCD
            bv = xv;
            bk = r;
        }
        wave_lexmin63(bv, bk);
        const float cmin = wave_min63(c);
        const bool any_viol = __builtin_amdgcn_ballot_w64(viol != 0) != 0;
        if (lane == 63) {
            uint64_t* part = x.part + ((size_t)q * x.G + rg) * 2;
            g_st64(part, ((uint64_t)(any_viol ? 1u : 0u) << 32) | __builtin_bit_cast(uint32_t, cmin));
            g_st64(part + 1, lex_key(bv, bk));
#if SVH_DIAG_AB == 7  // diagnostics: no arrival count (the last range combines, unordered)
            last = rg == NR - 1 ? 1u : 0u;
#else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t d = __hip_atomic_fetch_add(x.done + (size_t)q * SVH_DIAG_DONE_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = d == NR - 1 ? 1u : 0u;
#endif
#if SVH_DIAG_AB == 8  // diagnostics: the arrival count, no combine
            last = 0;
#endif
        }
        last = readlane_u(last, 63);
    }
    if (last) {  // this wave combines sequence q: lanes read the ranges' partials
        float C = kInf, bv2 = kInf;
        uint32_t bk2 = kNoRow, vi = 0;
        for (uint32_t u = lane; u < NR; u += 64) {
            const uint64_t* pu = x.part + ((size_t)q * x.G + u) * 2;
            const uint64_t a = g_ld64(pu), k2 = g_ld64(pu + 1);
            C = fminf(C, __builtin_bit_cast(float, (uint32_t)a));
            vi |= (uint32_t)(a >> 32);
            if (k2 != ~0ull) lex_min(bv2, bk2, lex_key_value(k2), lex_key_index(k2));
        }
        C = wave_min63(C);
        wave_lexmin63(bv2, bk2);
        const bool any = __builtin_amdgcn_ballot_w64(vi != 0) != 0;
        if (lane == 63) {
            float* out = b.scores + (size_t)q * m.n;
            if (m.rowF >= 0) {
                out[m.rowF] = F;
                lex_min(bv2, bk2, F, (uint32_t)m.rowF);
            }
            if (m.rowS >= 0) {
                out[m.rowS] = C;
                lex_min(bv2, bk2, C, (uint32_t)m.rowS);
            }
            if (b.best) b.best[q] = bk2 == kNoRow ? -1 : (int64_t)bk2;
            x.viol[q] = any ? 1u : 0u;
            __hip_atomic_store(x.done + (size_t)q * SVH_DIAG_DONE_STRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (any) rrow[w] = q;
        }
    }
    // rows whose speculation failed: re-run exactly by this workgroup (pipe_rerun_row, the latency
    // plan's serial recurrence with F's light term restored) -- no second launch on the common path
    __syncthreads();
    uint32_t rq[W];  // read before any re-run: its scores overwrite this part of the LDS
#pragma unroll
    for (int u = 0; u < W; ++u) rq[u] = rrow[u];
#pragma unroll
    for (int u = 0; u < W; ++u) {
        if (rq[u] != kNoRow) {
            __syncthreads();
            pipe_rerun_row<2, W, SX>(m, b, rq[u], lds);
        }
    }
}

// One workgroup per row after the main launch: the row's NR partials -> S, best state, the
// violation flag; a row whose speculation failed is re-run here exactly (pipe_rerun_row).
template <bool SX>
__global__ __launch_bounds__(256) void diag_finish_kernel(PipeModel m, FusedBatch b, PipeScratch x) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u;
    uint32_t* flag = reinterpret_cast<uint32_t*>(lds + 2 * (size_t)m.P + 8);
    if (tid < 64) {
        float C = kInf, bv = kInf;
        uint32_t bk = kNoRow, vi = 0;
        for (uint32_t u = lane; u < m.nrng; u += 64) {
            const uint64_t* pu = x.part + ((size_t)q * x.G + u) * 2;
            const uint64_t a = pu[0], k2 = pu[1];
            C = fminf(C, __builtin_bit_cast(float, (uint32_t)a));
            vi |= (uint32_t)(a >> 32);
            if (k2 != ~0ull) lex_min(bv, bk, lex_key_value(k2), lex_key_index(k2));
        }
        C = wave_min63(C);
        wave_lexmin63(bv, bk);
        const bool any = __builtin_amdgcn_ballot_w64(vi != 0) != 0;
        if (lane == 63) {
            float* out = b.scores + (size_t)q * m.n;
            if (m.rowF >= 0) lex_min(bv, bk, out[m.rowF], (uint32_t)m.rowF);
            if (m.rowS >= 0) {
                out[m.rowS] = C;
                lex_min(bv, bk, C, (uint32_t)m.rowS);
            }
            if (b.best) b.best[q] = bk == kNoRow ? -1 : (int64_t)bk;
            x.viol[q] = any ? 1u : 0u;
            *flag = any ? 1u : 0u;
        }
    }
    __syncthreads();
    if (*flag) pipe_rerun_row<2, 4, SX>(m, b, q, lds);
}

template <int W>
const void* diag_ptr(bool sx) {
    return sx ? reinterpret_cast<const void*>(&diag_viterbi_kernel<W, true>)
              : reinterpret_cast<const void*>(&diag_viterbi_kernel<W, false>);
}

}  // namespace

uint32_t diag_waves_for(uint64_t nseq) { return nseq >= 4 ? 4u : nseq >= 2 ? 2u : 1u; }

size_t diag_lds_bytes(uint32_t W, uint32_t S, uint32_t P) {
    const size_t rerun = (2 * (size_t)P + 2 * W) * 4;  // pipe_rerun_row: v[2][P], red[2][W]
    const size_t mainb = diag_lds_main(W, S);
    return mainb > rerun ? mainb : rerun;
}

hipError_t launch_diag(const PipeModel& m, const FusedBatch& b, const PipeScratch& x, hipStream_t stream) {
    if (!m.dtab || m.nrng == 0 || m.SM != 2 || m.S == 0 || m.S > kDMaxSym || (size_t)m.nrng * 64 > m.P || m.wide ||
        b.cmask || b.run_mask || (b.v_in && !b.v_in_row) || !x.part || !x.done || !x.viol || b.nseq > x.rows || x.G < m.nrng)
        return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    const uint32_t W = diag_waves_for(b.nseq);
    const void* fn = W == 4 ? diag_ptr<4>(m.sx != 0) : W == 2 ? diag_ptr<2>(m.sx != 0) : diag_ptr<1>(m.sx != 0);
    size_t lds = diag_lds_bytes(W, m.S, m.P);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    const uint64_t grid = ((uint64_t)b.nseq + W - 1) / W * m.nrng;
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    // even placement: a launch that fits the chip gets its LDS request raised so that no CU can take
    // more than ceil(grid / CUs) of its workgroups (the dispatcher would otherwise stack up to four
    // on some CUs and leave others empty; the kernel ends with its most loaded CU)
    if (m.cus) {
        const uint64_t per_cu = (grid + m.cus - 1) / m.cus;
        if (per_cu * lds <= 160 * 1024) {
            const size_t cap = (160 * 1024 / per_cu) & ~(size_t)511;
            lds = cap > lds ? cap : lds;
        }
    }
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    PipeModel mm = m;
    FusedBatch bb = b;
    PipeScratch xx = x;
    void* args[] = {&mm, &bb, &xx};
    const hipError_t e = hipLaunchKernel(fn, dim3((uint32_t)grid), dim3(64 * W), args, lds, stream);
#if SVH_DIAG_FINISH
    if (e != hipSuccess) return e;
    const void* fin = m.sx ? reinterpret_cast<const void*>(&diag_finish_kernel<true>)
                           : reinterpret_cast<const void*>(&diag_finish_kernel<false>);
    return hipLaunchKernel(fin, dim3(b.nseq), dim3(256), args, (2 * (size_t)m.P + 8 + 1) * 4, stream);
#else
    return e;
#endif
}

}  // namespace svh
