// Pipelined chain Viterbi kernel (gfx950): the latency path for MSV-shaped models whose feeder row
// F (N) is speculated and verified exactly (kernels.h, PipeModel).
//
// Reference hot loop: Viterbi_impl/GraphBLAS_impl.cpp:59-73 (same association, bit-identical):
//     v'[j] = min_k fl( fl(E[o][j] + T^T[j][k]) + v[k] )
// For the light rows of the chain shape this is v'_p = min(fl(eb_p(o) + v_{p-1}), fl(ea_p(o) + F))
// with eb_p(o) = fl(E_o[p] + bw_p), ea_p(o) = fl(E_o[p] + aw_p) (the reference's first add, folded
// into the table), so once F's sequence is known a position depends only on its chain predecessor
// one observation earlier: a wavefront over (position block, observation) with no feedback.
//
// Geometry: block b = 64*SM consecutive positions, one wave (lane l holds positions
// b*64*SM + l*SM + s); W blocks per workgroup, G = ceil(nblk / W) workgroups per sequence.
// Each wave sweeps all observations of its block.  Its last position's score of observation t
// is the chain input of the next block's position 0 at t+1:
//   * within a workgroup: every lane writes its score into an LDS ring [kPipeRing][64] each
//     observation; the wave publishes "observations done" once per group of 8; the consumer
//     waits for the whole group, reads its 8 boundary values with one ds_read and extracts them
//     with v_readlane (one per observation); producers check the consumer's count once per
//     group before reusing ring slots.
//   * between workgroups: the last wave stores 8-byte granules {score, tag} (agent scope, sc1)
//     into a ring of kPipeGRing per sequence boundary; the next workgroup's first wave keeps
//     kPipeAhead groups of granule loads in flight and checks the tags; flow control through a
//     tagged progress word.  Workgroups take dynamic tickets in start order, so a consumer's
//     producer always started first (no deadlock when the grid exceeds residency).
// Per lane and observation the heavy side is: S partial  c' = min(fl(A_S + m), fl(X_SS + c)
// [, fl(X_SF + F)]) with m = min of the lane's scores at t-1 (exact: S(t) = min over lanes of c,
// fl(a + .) is monotone), F' = fl(X_FF + F), and the check fl(A_F + m) < F' (a violation: F
// would have taken its light term, the speculation and everything after it is void).
// The last workgroup of a sequence to finish combines the partials (S, argmin, violation).
//
// Decoded paths (PATHS = 1, 2): per observation and light position the "took F's term" bit
// (compare into VCC + v_addc into a per-lane word per slot, stored every 32 observations; PATHS 2
// when F wins every tie: one compare), per observation the lane's {light minimum of t-1, sink
// partial of t} into an LDS ring that the wave folds every 32 observations into per-half-wave
// partial records (transposed: lane l reduces row l % 32 over its half), light-score checkpoints
// every kCkptEvery observations and F every 32 (block 0).  pipe_paths.hip turns these into the
// heavy records and walks the paths.
#pragma once
#include "pipe_common.h"

namespace svh {

using namespace dev;
using namespace pipe_dev;

namespace {

typedef float f32x32 __attribute__((ext_vector_type(32)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr uint32_t kR = kPipeRing;

// Granule hand-off between workgroups: groups of 8 granules the consumer keeps in flight ahead of
// use (1, 2 or 4), and the step of the next group at which the producer stores a finished group's
// granules (0: at the end of the next group).  A/B knobs (tools/ab_build.sh -D...).
#ifndef SVH_PIPE_GPF
#define SVH_PIPE_GPF 2
#endif
#ifndef SVH_PIPE_GST
#define SVH_PIPE_GST 2
#endif
constexpr uint32_t kGpf = SVH_PIPE_GPF;
// (Round 5, measured and not kept: four groups for a consumer whose producer sits on another XCD.
// The cross-XCD rows, 2 of the headline's 50, end the launch 15-25 us after the XCD-local ones; with
// four groups in flight their prefetches outran the producer and polled: 0.296-0.306 ms against
// 0.250-0.254, profiles/r05_s8.)
constexpr uint32_t kGst = SVH_PIPE_GST;
static_assert(kGpf == 1 || kGpf == 2 || kGpf == 4, "granule prefetch depth");
static_assert(kGst < 8, "granule store step");

// LDS boundary ring layout: 0 = [u][lane] (every step stores its row, one ds_write_b32; TM = 0,
// pipe.hip); 1 = [u / 8][lane][u % 8]: a group's 8 last-slot scores stay in registers and go out as
// two ds_write_b128 per group (the consumer reads lane 63's 8 values as one contiguous 32 bytes;
// TM = 1 / 2, pipe_tm1.hip and pipe_tm1p.hip define it).
#ifndef SVH_PIPE_RING8
#define SVH_PIPE_RING8 0
#endif
// ring slot of cycle position u (0..31) and lane l
__device__ __forceinline__ uint32_t ring_idx(uint32_t u, uint32_t l) {
    return SVH_PIPE_RING8 ? ((u >> 3) * 64 + l) * 8 + (u & 7u) : u * 64 + l;
}

template <uint32_t N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N < 64, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS reads of the exchange kept where they are issued (A/B knob SVH_PIPE_LDSX, default 1; within
// run-to-run noise on the headline, 0.258-0.265 vs 0.256-0.264 ms, profiles/r04_s9/ab.log): the
// compiler otherwise (a) hoisted the slow path's re-load of the next group's boundary vector out of
// its branch, so every group re-read it at its first use and waited for it there, and (b) moved the
// readfirstlane of the neighbours' counts (read four steps before their use) up to the reads,
// waiting for them at once.  An opaque zero in the slow path's address and an asm use of each count
// where it is needed keep both reads' latency behind steps.
#ifndef SVH_PIPE_LDSX
#define SVH_PIPE_LDSX 1
#endif

// XCD-local hand-offs (A/B knob SVH_PIPE_XL): every workgroup publishes its XCC id; a granule
// producer whose consumer workgroup sits on the same XCD stores its granules with plain stores
// (kept in the XCD's L2) instead of agent-scope write-through stores (which drop the line, so the
// consumer's L2-served load goes to the fabric), and a consumer on its producer's XCD does the same
// with its progress word.  The reading side is unchanged (agent-scope loads: L1 bypassed, served
// by the L2 the plain store wrote); a pair on different XCDs, or one whose id is not known yet,
// keeps write-through stores.  Measured on the headline: 0.248-0.251 ms against 0.258-0.265
// (profiles/r04_s9/ab.log); the XCD half whose hops were slow (§5f) comes down to the other's rate.
#ifndef SVH_PIPE_XL
#define SVH_PIPE_XL 1
#endif

// The next group's boundary vector (SRC 1) read at step 4, right after the producer's count it is
// validated against (A/B knob SVH_PIPE_EARLYV): LDS executes one CU's instructions in order and the
// producer wrote its ring before its count, so a count that covers the group guarantees the vector
// read issued after it sees the group; otherwise the slow path waits and reads it again.  At the
// group's end (0) the read's latency sat in front of the next group's second step.
#ifndef SVH_PIPE_EARLYV
#define SVH_PIPE_EARLYV 1
#endif

// Exchange helpers (A/B knob SVH_PIPE_XHELP, workgroups of three waves or more): the vector-memory
// counter retires a wave's loads and stores in issue order, so a wave that both stores to another
// XCD (write-through, acknowledged late) and waits for a load waits for those stores too.  The
// granule reader (wave 0) published its progress word and the granule writer (wave W - 1) loaded
// its consumer's, so on the rows whose hops cross XCDs both waited on remote stores every 32
// observations.  With the helpers wave 1, which has no other global traffic, publishes the progress
// (its own, never ahead of wave 0's) and wave W - 2 loads the consumer's word once per 32
// observations into an LDS slot that wave W - 1 reads: wave 0 only loads and wave W - 1 only stores.
#ifndef SVH_PIPE_XHELP
#define SVH_PIPE_XHELP 1
#endif

// Step of a group at which the neighbours' counts (and, SVH_PIPE_EARLYV, the next group's vector)
// are read (A/B knob SVH_PIPE_CNTSTEP, 1..7): later reads see a producer further ahead, so the next
// group's vector is valid more often, at the price of less time to hide the LDS latency.  Headline
// kernel (profiles/r05_xhelp/ab_cntstep.log): step 4 0.2296-0.2329 ms, 5 0.2283-0.2291, 6
// 0.2284-0.2295, 7 0.243-0.252 (the read's latency no longer hidden).
#ifndef SVH_PIPE_CNTSTEP
#define SVH_PIPE_CNTSTEP 5
#endif
// (Round 5, measured and not kept: the pair tables' compiler barrier placed after the prologue's
// other loads, so the heavy constants, the first state and the symbol windows load while the tables
// are in flight.  The first sweep started later, not earlier (7.2 us after the launch's first entry
// against 5.9), and the kernel ran 0.2291-0.2301 ms against 0.2272-0.2289,
// profiles/r05_xhelp/ab_lateopq.log.)
// (Round 5, measured and not kept: the slow path's count and vector reads issued together, one
// LDS round trip instead of two.  Waves 1-2 of the workgroups fed by granules take that path in
// 43-67% of their groups; with it cheaper they ran closer to their producer and took it more often
// (78-97%), for the same kernel time: 0.2300-0.2318 ms against 0.2304-0.2322,
// profiles/r05_xhelp/ab_slow1.log.)
// (Round 5, measured and not kept: a granule consumer's first boundary awaited alone instead of
// with the producer's whole first group.  The sweeps start earlier but the rows end no sooner (the
// workgroup hop's lag is set by the groups' hand-off, not by the start) and the early prefetches
// poll: 0.2307-0.2323 ms against 0.2291-0.2299, profiles/r05_xhelp/ab_gfirst.log.)
static_assert(SVH_PIPE_CNTSTEP >= 1 && SVH_PIPE_CNTSTEP <= 7, "count step");

// Diagnostic ablation (-DSVH_PIPE_NOWAIT, timing only, wrong results): every exchange operation
// runs, but no wait on a neighbour does (counts, flow control, granule tags and progress words are
// taken as ready): the rate of a wave when no neighbour ever holds it up.
#ifdef SVH_PIPE_NOWAIT
constexpr bool kNoWait = true;
#else
constexpr bool kNoWait = false;
#endif
// Diagnostic ablation (-DSVH_PIPE_NOPSTORE, timing only, wrong paths): the path variant computes
// and folds its records but stores none of them (tie masks, checkpoints, folded records) to HBM.
#ifdef SVH_PIPE_NOPSTORE
constexpr bool kNoPStore = true;
#else
constexpr bool kNoPStore = false;
#endif
// Diagnostic ablations (timing only, wrong paths): -DSVH_PIPE_NOFOLD skips the fold of the record
// ring every 32 observations; -DSVH_PIPE_NOPRING also skips the ring's stores (the step's records).
#ifdef SVH_PIPE_NOFOLD
constexpr bool kNoFold = true;
#else
constexpr bool kNoFold = false;
#endif
#ifdef SVH_PIPE_NOPRING
constexpr bool kNoPRing = true;
#else
constexpr bool kNoPRing = false;
#endif

// Slow-path loads that wait for themselves (SVH_PIPE_SYNCSLOW, default 1): the compiler tracks every
// load it emits, so a poll loop's reload left pending where the slow path rejoins the body made it
// drain every outstanding operation there -- on the fast path too: the granule consumer's body then
// waited with vmcnt(0) for the next group's prefetch once per group, and the LDS consumers'
// re-read of a boundary vector forced an lgkmcnt wait behind the ring stores.  A load whose wait is
// inside its own asm leaves nothing for the compiler to drain (the wide kernel's g_ld64_sync).
#ifndef SVH_PIPE_SYNCSLOW
#define SVH_PIPE_SYNCSLOW 1
#endif
__device__ __forceinline__ uint64_t g_ld64_slow(const uint64_t* p) {
    if constexpr (SVH_PIPE_SYNCSLOW) {
        uint64_t r;
        asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
        return r;
    }
    return g_ld64(p);
}
__device__ __forceinline__ uint32_t lds_ld32_slow(const uint32_t* p) {
    if constexpr (SVH_PIPE_SYNCSLOW) {
        uint32_t r;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_addr(p)) : "memory");
        return r;
    }
    return lds_ld32(p);
}
__device__ __forceinline__ float lds_ldf_slow(const float* p) {
    if constexpr (SVH_PIPE_SYNCSLOW) {
        float r;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(lds_addr(p)) : "memory");
        return r;
    }
    return *p;
}

// One lane's LDS store of a wave-uniform word (a wave's count): EXEC narrowed to lane 0 inside the
// asm (no divergent branch in the compiler's view).  Measured and not kept (round 4): every lane
// storing, lanes 1..63 into a sink of their own (no EXEC writes), within noise.
__device__ __forceinline__ void lds_put1(uint32_t addr, uint32_t v) {
    uint64_t saved;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "s_nop 1\n\t"
        "ds_write_b32 %1, %2\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "v"(addr), "v"(v)
        : "memory");
}

// The chain term of slot 0 alone (TM = 2, whose feeder terms come out of the indexed block):
// xb = fl(eb + (lane ? x[lane-1] : b)), b the SGPR boundary (R < 0), lane 0 of bvv (R = 0) or lane R
// of bvv (row_ror:16-R).  x was written before the step's indexed block and bvv at the start of
// the group, so both DPP reads have their wait states (tools/dpp_hazards.py checks every build).
template <int R>
__device__ __forceinline__ float chain_b(float eb, float b, float x) {
    float xb;
    if constexpr (R < 0) {
        asm("v_add_f32_e32 %0, %1, %2\n\t"
            "v_add_f32_dpp %0, %3, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb)
            : "s"(b), "v"(eb), "v"(x));
    } else if constexpr (R == 0) {
        asm("v_add_f32_e32 %0, %1, %2\n\t"
            "v_add_f32_dpp %0, %3, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb)
            : "v"(b), "v"(eb), "v"(x));
    } else {
        asm("v_add_f32_dpp %0, %1, %2 row_ror:%4 row_mask:0xf bank_mask:0xf\n\t"
            "v_add_f32_dpp %0, %3, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb)
            : "v"(b), "v"(eb), "v"(x), "n"(16 - R));
    }
    return xb;
}

// Chain and feeder terms of slot 0: xb = fl(eb + (lane ? x[lane-1] : bnd)), xa = fl(ea + f).
// The DPP read of x follows two VALU instructions of this block (its two wait states).
__device__ __forceinline__ void chain_terms(float& xb, float& xa, float eb, float ea, float bnd, float f,
                                            float x) {
    asm("v_add_f32_e32 %0, %2, %3\n\t"
        "v_add_f32_e32 %1, %4, %5\n\t"
        "v_add_f32_dpp %0, %6, %3 wave_shr:1 row_mask:0xf bank_mask:0xf"
        : "=&v"(xb), "=&v"(xa)
        : "s"(bnd), "v"(eb), "v"(f), "v"(ea), "v"(x));
}

// The same with lane 0's chain input taken from lane R of the group vector bvv (row_ror:16-R
// rotates lane R of each row of 16 into its lane 0; no SGPR round trip).  xa comes first, so x
// has its two wait states inside the block; bvv has one inside the block and gets the other from
// the schedule around it (bvv is written at the start of a group, never by the instruction before
// a step).  The compiler does not see DPP inside asm, so the build checks every DPP read of the
// kernel for the two wait states (tools/dpp_hazards.py, Makefile); the s_nop the block carried
// before cost 1.6 % (A/B 0.361 vs 0.367 ms).
template <int R>
__device__ __forceinline__ void chain_terms_v(float& xb, float& xa, float eb, float ea, float bvv, float f,
                                              float x) {
    if constexpr (R == 0) {
        asm("v_add_f32_e32 %1, %4, %5\n\t"
            "v_add_f32_e32 %0, %2, %3\n\t"
            "v_add_f32_dpp %0, %6, %3 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb), "=&v"(xa)
            : "v"(bvv), "v"(eb), "v"(f), "v"(ea), "v"(x));
    } else {
        asm("v_add_f32_e32 %1, %4, %5\n\t"
            "v_add_f32_dpp %0, %2, %3 row_ror:%7 row_mask:0xf bank_mask:0xf\n\t"
            "v_add_f32_dpp %0, %6, %3 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb), "=&v"(xa)
            : "v"(bvv), "v"(eb), "v"(f), "v"(ea), "v"(x), "n"(16 - R));  // lane 0 <- lane R
    }
}

// TM 3: both feeder terms in one packed add, xa = {ea_0 + F, ea_1 + F} (F = the high half of cf),
// then slot 0's chain term as chain_terms / chain_terms_v (the packed add and, R < 1, the plain add
// give the DPP read of x its two wait states inside the block).
template <int R>
__device__ __forceinline__ void chain_terms_pk(float& xb, f2& xa, f2 ea, float eb, float bnd, f2 cf, float x) {
    if constexpr (R < 0) {
        asm("v_pk_add_f32 %1, %3, %5 op_sel:[0,1] op_sel_hi:[1,1]\n\t"
            "v_add_f32_e32 %0, %2, %4\n\t"
            "v_add_f32_dpp %0, %6, %4 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb), "=&v"(xa)
            : "s"(bnd), "v"(ea), "v"(eb), "v"(cf), "v"(x));
    } else if constexpr (R == 0) {
        asm("v_pk_add_f32 %1, %3, %5 op_sel:[0,1] op_sel_hi:[1,1]\n\t"
            "v_add_f32_e32 %0, %2, %4\n\t"
            "v_add_f32_dpp %0, %6, %4 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb), "=&v"(xa)
            : "v"(bnd), "v"(ea), "v"(eb), "v"(cf), "v"(x));
    } else {
        asm("v_pk_add_f32 %1, %3, %5 op_sel:[0,1] op_sel_hi:[1,1]\n\t"
            "v_add_f32_dpp %0, %2, %4 row_ror:%7 row_mask:0xf bank_mask:0xf\n\t"
            "v_add_f32_dpp %0, %6, %4 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb), "=&v"(xa)
            : "v"(bnd), "v"(ea), "v"(eb), "v"(cf), "v"(x), "n"(16 - R));  // lane 0 <- lane R
    }
}

// Table reads of a step (template TM):
//   0  per-slot tables f32x32 [SM][eb|ea] (symbol o in register o): the compiler's indexed moves,
//      one s_set_gpr_idx block of SM x 2 v_mov, and the heavy constants by four v_readlane;
//   1  (SM = 2, at most kPairSym symbols) four pair-interleaved tables pinned to v2..v161,
//      register 2o + u = value u of symbol o: T1 = {eb_0, ea_0}, T2 = {eb_1, ea_1},
//      T3 = {A_S, A_F}, T4 = {X_SS, X_FF}; one idx block of four v_mov_b64 (M0 = 2o, the symbol
//      windows are loaded pre-doubled), so no v_readlane and no SGPR hand-off per step;
//   2  the same tables read as M0-indexed operands of the adds that use them (one gpr_idx(SRC0)
//      block, only eb_0 moved out for slot 0's DPP chain add);
//   3  as 1 with T1 = {ea_0, ea_1}, T2 = {eb_0, eb_1}: both feeder terms come out of one
//      v_pk_add_f32 with F broadcast from the high half of the {C, F} pair (op_sel), one VALU less;
//   4  as 2 with the layout of 3 (the packed feeder add reads T1 as an indexed 64-bit operand).
// tools/ubench/step_ubench.hip prices the two at 158 vs 101 shader cycles per observation (no
// exchange, 4 waves per CU).  Measured and not kept (round 3): every table and constant read as an
// M0-indexed operand of the add that uses it (13 VALU, 66 vs 72 ns a step, 1 % in the pipeline);
// indexed adds through gpr_idx(SRC0) with the DPP pair after the block (0.39 ms), everything but the
// constants through gpr_idx(SRC1) (0.37), the constants by a broadcast ds_read_b128 a step ahead
// instead of v_readlane (0.38).
constexpr uint32_t kPairSym = kPairSymbols;
typedef float f32x8 __attribute__((ext_vector_type(8)));

// Slot 0's chain input for a step: R < 0 the uniform boundary b (SGPR, single observations),
// R = 0 lane 0 of the group vector, R = 1..7 lane R of the group vector (row_ror:16-R).
template <int R>
struct ChainIn {
    static constexpr int value = R;
    float b;
};

// Lanes 1..63 take v of lane - 1 (DPP wave_shr:1); lane 0 takes lane R of bvv (row_ror:16-R; R = 0:
// lane 0's own bvv, which is also the form for a uniform boundary).  Built from the DPP builtins, so
// the compiler inserts the wait states (the level-2 step, L2 below).
template <int R>
__device__ __forceinline__ float shr_in(float v, float bvv) {
    int old = __builtin_bit_cast(int, bvv);
    if constexpr (R > 0) old = __builtin_amdgcn_update_dpp(old, old, 0x120 + (16 - R), 0xf, 0xf, false);
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(old, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, false));
}


// Exact serial re-run of row q whose speculation failed (m.rerun: the scores variant of the latency
// plan, P small enough for the ring's LDS), by the workgroup that combines the row, so that no
// second launch is needed on the common path (round 5 launched the serial chain kernel after every
// pass, 4.1 us of 50 workgroups that exit at once).  The recurrence is the one the sweep speculates
// on, with F's light term restored (GraphBLAS_impl.cpp:64-73, the association of chain_impl.h):
//   v'_p = min(fl(eb_p(o) + v_{p-1}), fl(ea_p(o) + F)),   F' = min(fl(A_F + mu), fl(X_FF + F)),
//   C'   = min(fl(A_S + mu), fl(X_SS + C) [, fl(X_SF + F)]),   mu = min_p v_p (scores of t-1).
// Scores double-buffered in LDS (v[2][P], position-major), thread i updates positions i, i + T, ...
// (the table reads coalesce), per-wave minima in red[2][W]; one barrier per observation.  Slow
// (~2 us per observation) but only for rows that fail the check, which no reference workload does.
template <int SM, int W, bool SX>
__device__ __forceinline__ void pipe_rerun_row(const PipeModel& m, const FusedBatch& b, uint32_t q, float* lds) {
    constexpr uint32_t T = 64 * W;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t P = m.P, S = m.S;
    float* vb = lds;                       // [2][P]
    float* red = lds + 2 * P;              // [2][W]
    const uint8_t* __restrict__ sym = b.symbols + b.sym_off[q];
    const uint32_t len = (uint32_t)uniform((int)b.end[q]);
    const uint32_t beg = (uint32_t)uniform((int)b.begin[q]);
    const uint32_t first = beg ? beg : 1u;
    float F, C;
    float mu = kInf;
    // state at observation first - 1
    if (beg == 0) {
        const uint32_t o0 = sym[0];
        for (uint32_t p = tid; p < P; p += T) {
            const float v = m.e0[(size_t)o0 * P + p] + m.start[p];
            vb[p] = v;
            mu = fminf(mu, v);
        }
        F = m.rowF >= 0 ? m.hc[o0 * 8 + 5] + m.startF : kInf;
        C = m.rowS >= 0 ? m.hc[o0 * 8 + 6] + m.startS : kInf;
    } else {
        const float* vin = b.v_in + (size_t)b.v_in_row[q] * m.n;
        for (uint32_t p = tid; p < P; p += T) {
            const uint32_t r = m.lrow[p];
            const float v = r != kNoRow ? vin[r] : kInf;
            vb[p] = v;
            mu = fminf(mu, v);
        }
        F = m.rowF >= 0 ? vin[m.rowF] : kInf;
        C = m.rowS >= 0 ? vin[m.rowS] : kInf;
    }
    mu = wave_min63(mu);
    if (lane == 63) red[w] = mu;
    __syncthreads();
    uint32_t cur = 0;
    for (uint32_t t = first; t < len; ++t) {
        const uint32_t o = (uint32_t)uniform((int)sym[t]);
        float m0 = kInf;
#pragma unroll
        for (int u = 0; u < W; ++u) m0 = fminf(m0, red[cur * W + u]);
        const float4 h = *reinterpret_cast<const float4*>(m.hc + o * 8);  // A_S A_F X_SS X_FF
        const float Fn = fminf(h.y + m0, h.w + F);
        float Cn = fminf(h.x + m0, h.z + C);
        if constexpr (SX) Cn = fminf(Cn, m.hc[o * 8 + 4] + F);
        const float* vc = vb + cur * P;
        float* vn = vb + (cur ^ 1u) * P;
        float mn = kInf;
        for (uint32_t p = tid; p < P; p += T) {
            // position p = (blk, lane l, slot s) of the sweep's layout: tab[((blk S + o) SM + s) 64 + l]
            const uint32_t blk = p / (64 * SM), r = p - blk * 64 * SM, l = r / SM, s = r - l * SM;
            const float2 e = m.tab[((size_t)(blk * S + o) * SM + s) * 64 + l];
            const float prev = p ? vc[p - 1] : kInf;
            const float v = fminf(e.x + prev, e.y + F);
            vn[p] = v;
            mn = fminf(mn, v);
        }
        mn = wave_min63(mn);
        if (lane == 63) red[(cur ^ 1u) * W + w] = mn;
        F = Fn;
        C = Cn;
        cur ^= 1u;
        __syncthreads();
    }
    // scores, best state (lexicographic (value, row) argmin, lowest row on ties)
    float* out = b.scores + (size_t)q * m.n;
    const float* vc = vb + cur * P;
    float bv = kInf;
    uint32_t bk = kNoRow;
    for (uint32_t p = tid; p < P; p += T) {
        const uint32_t r = m.lrow[p];
        if (r != kNoRow) {
            out[r] = vc[p];
            lex_min(bv, bk, vc[p], r);
        }
    }
    wave_lexmin63(bv, bk);
    __syncthreads();  // every wave has read vc and red
    if (lane == 63) {
        red[2 * w] = bv;
        red[2 * w + 1] = __builtin_bit_cast(float, bk);
    }
    __syncthreads();
    if (tid == 0) {
        float v2 = kInf;
        uint32_t k2 = kNoRow;
        for (uint32_t u = 0; u < (uint32_t)W; ++u) lex_min(v2, k2, red[2 * u], __builtin_bit_cast(uint32_t, red[2 * u + 1]));
        if (m.rowF >= 0) {
            out[m.rowF] = F;
            lex_min(v2, k2, F, (uint32_t)m.rowF);
        }
        if (m.rowS >= 0) {
            out[m.rowS] = C;
            lex_min(v2, k2, C, (uint32_t)m.rowS);
        }
        if (b.best) b.best[q] = k2 == kNoRow ? -1 : (int64_t)k2;
    }
}

// FLOOR (svh_batch_step_floor_ms): every wave sweeps its block as block 0 does -- no boundary input,
// no exchange, no waits -- so the launch times the step alone (the per-observation issue floor of
// one wave); its scores are meaningless and go to a scratch buffer.
template <int SM, int W, bool SX, int PATHS, int TM, bool L2 = false, bool FLOOR = false>
__global__ __launch_bounds__(64 * W) void pipe_viterbi_kernel(PipeModel m, FusedBatch b, PipeScratch x) {
    static_assert(TM == 0 || SM == 2, "pair tables: two slots per lane");
    static_assert(TM >= 0 && TM <= 4, "table mode");
    static_assert(!L2 || (SM == 2 && TM == 4 && PATHS == 0 && SVH_PIPE_RING8), "level 2: the pair-table scores kernel");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* ring = lds;                                                  // [W][kR][64]
    uint32_t* cnt = reinterpret_cast<uint32_t*>(ring + W * kR * 64);    // [16]
    float* ctab = reinterpret_cast<float*>(cnt + 16);                   // [S][8]
    float* red = ctab + m.S * 8;                                        // [W][4]
    uint32_t* tick = reinterpret_cast<uint32_t*>(red + W * 4);
    // PATHS: [W][8 quads][kPQuadStride] {pm, c} of 4 observations per lane, 16-byte aligned after the rest
    float* pring = lds + (pipe_lds_bytes(W, m.S) + 15) / 16 * 4;

    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t w = (uint32_t)uniform((int)(tid >> 6));
    const uint32_t S = m.S, P = m.P, G = m.G;
    // (row, workgroup) of this workgroup, from a ticket taken in start order, so a consumer's
    // producer has always started before it (no deadlock when the grid exceeds residency or other
    // launches hold CUs).  Default: one ticket counter, rows in ticket order.  x.xmap (the runtime
    // sets it when the launch fits the chip at one workgroup per CU, the grid padded to a multiple
    // of 8): per-class tickets, so that a row's G workgroups share an XCD class (blocks b and b + 8
    // share an XCD under the observed round-robin placement; speed only -- the hand-offs check the
    // real XCC ids, SVH_PIPE_XL).  Every class r = b % 8 holds n = N / 8 blocks and takes f = n / G
    // rows whole: its k-th ticket (k < f G) is member k % G of row r f + k / G, members numbered in
    // start order.  The n - f G spare tickets of the classes form the remaining rows from one more
    // counter, also in start order (slot u is member u % G of row 8 f + u / G), so every member's
    // producer has started before it, whatever the residency.  Those rows span XCDs; with the
    // exchange helpers their hops cost no more than the others' (class-ordered spare slots, which
    // kept them to two XCD changes but numbered members across classes out of start order, measured
    // the same: profiles/r05_xhelp/ab_leftover_start_order.log).  Slots and rows past the batch are
    // dummies that only count themselves finished.
    if (tid == 0) {
        uint32_t t;
        if (x.xmap) {
            const uint32_t n = gridDim.x >> 3, r = blockIdx.x & 7u, f = n / G;
            const uint32_t k = __hip_atomic_fetch_add(x.ctr + kCtrClass + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (k < f * G) {
                t = (r * f + k / G) * G + k % G;
            } else {
                const uint32_t u = __hip_atomic_fetch_add(x.ctr + kCtrLeft, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                t = (8 * f + u / G) * G + u % G;
            }
        } else {
            t = __hip_atomic_fetch_add(x.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        *tick = t;
    }
    if (tid < 16) cnt[tid] = 0;
    for (uint32_t i = tid; i < S * 8; i += 64 * W) ctab[i] = m.hc[i];
    __syncthreads();
    const uint32_t id = (uint32_t)uniform((int)*tick);
    const uint32_t q = id / G, g = id - q * G;
    if (q >= b.nseq) {  // x.xmap: a padding slot of the grid (no row); counts itself finished
        if (tid == 0) {
            const uint32_t f = __hip_atomic_fetch_add(x.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (f == gridDim.x - 1) pipe_reset_counters(x);
        }
        return;
    }
    const uint32_t ep = (uint32_t)uniform((int)__hip_atomic_load(x.ctr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
#if SVH_PIPE_XL
    const uint32_t my_xcc = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xFu;  // hwreg(HW_REG_XCC_ID, 0, 4)
    if (tid == 0 && x.xcc)
        __hip_atomic_store(x.xcc + (size_t)q * G + g, (ep << 4) | my_xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif

    const uint8_t* __restrict__ sym = b.symbols + b.sym_off[q];
    // L2: the sweep's t runs over observations 1 .. 2 nch of the nch = (L - 1) / 2 chunks (every row
    // starts at observation 0; the odd tail is the step kernel's, runtime.cpp)
    const uint32_t len = L2 ? 1u + (((uint32_t)uniform((int)b.end[q]) - 1u) & ~1u) : (uint32_t)uniform((int)b.end[q]);
    const uint32_t beg = L2 ? 0u : (uint32_t)uniform((int)b.begin[q]);
    const uint32_t first = beg ? beg : 1u;  // first observation the steps run (state at first-1)
    const uint32_t blk = g * W + w;
    const bool act = blk < m.nblk;
    const bool lastb = blk + 1 >= m.nblk;
    // boundary roles: source 0 none (block 0), 1 LDS (previous wave), 2 granules (previous
    // workgroup); sink 0 none (last block), 1 LDS, 2 granules
    const int src = blk == 0 ? 0 : (w > 0 ? 1 : 2);
    const int dst = lastb ? 0 : (w + 1 < (uint32_t)W ? 1 : 2);

    float v[SM];  // light scores of the lane's positions
    f2 CF;        // {S partial of this lane, F'} (one register pair: the packed heavy update)
    uint32_t viol = 0;  // per lane: steps whose check failed (a VGPR count: no VALU -> SALU hand-off)
    uint32_t spins = 0;
    // PATHS: the last 32 "took F's term" bits per slot (bit 0 = newest), the static tie masks
    // (PATHS 1), the lane's light minimum of the last step's input scores
    uint32_t macc[PATHS ? SM : 1] = {};
    uint64_t pmC[PATHS ? SM : 1] = {};
    float last_pm = kInf;
    // diagnostics: 0 loop cycles, 1 head cycles, 2 tail cycles, 3 slow re-reads waiting for the
    // previous wave, 4 ... for the next wave (flow control), 5 ... for granules, 6 ... for the
    // consumer's progress word, 7 body iterations, 8 .. 11 the 100 MHz real-time clock at wave
    // entry, sweep start, body end, sweep end, 12 the wave's XCC_ID << 32 | HW_ID (placement), 13
    // the real-time clock when the wave's tables have arrived, 14 groups whose boundary vector was
    // re-read after a wait (the next group's early read not validated).
    // Built only with -DSVH_PIPE_DIAG (tools/ab_build.sh;
    // then SVH_PIPE_DEBUG=1 at run time): the counters would otherwise hold SGPRs through the loop
    // in the production kernel, whose SGPRs are its scarcest register file.
    unsigned long long dg[kPipeStamps] = {};
#ifdef SVH_PIPE_DIAG
    const bool dbg = m.stamps != nullptr;
#define SVH_RT(k) (dg[k] = dbg ? __builtin_amdgcn_s_memrealtime() : 0ull)
#else
    constexpr bool dbg = false;
#define SVH_RT(k) ((void)0)
#endif
    SVH_RT(8);
#ifdef SVH_PIPE_DIAG
    if (dbg)  // hwreg(HW_REG_XCC_ID) and hwreg(HW_REG_HW_ID), 32 bits each
        dg[12] = ((unsigned long long)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                 (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif

    if (act) {
        const uint32_t p0 = blk * 64 * SM + lane * SM;
        // ---- tables: (eb, ea) of the lane's positions for every symbol, in VGPRs
        f32x32 EB[SM], EA[SM];
#pragma unroll
        for (int s = 0; s < SM; ++s)
#pragma unroll
            for (int o = 0; o < 32; ++o) {
                // unconditional loads (a clamped symbol), then a select: all 32 x SM loads go out
                // back to back (a conditional load per symbol serialised them: ~15 us of prologue)
                const uint32_t oc = (uint32_t)o < S ? (uint32_t)o : S - 1u;
                const float2 e = m.tab[((size_t)(blk * S + oc) * SM + s) * 64 + lane];
                EB[s][o] = (uint32_t)o < S ? e.x : kInf;
                EA[s][o] = (uint32_t)o < S ? e.y : kInf;
            }
        // mode 3: the pair-interleaved tables (symbols >= S: +inf)
        constexpr bool kT3 = TM >= 1;  // pair tables (symbols pre-doubled)
        constexpr bool kT4 = TM == 1 || TM == 3;  // ... read by four 64-bit moves
        constexpr int NT = 4;
        f32x32 TA[NT];
        f32x8 TB[NT];
        if constexpr (L2) {
            // level 2 (three pair tables, register 2o + u of table k = value u of symbol o):
            // T0 {eb_0, eb_1}, T1 {ea_0, ea_1}, T2 {eb, ea} of position p0 - 1 (lane - 1's slot 1, the
            // previous block's last position for lane 0; +inf before block 0).  The heavy constants
            // come from the lane tables by v_readlane: six pinned tables (240 registers) left the
            // step 14 of the 256 architectural VGPRs (the first build spilled 567 registers)
#pragma unroll
            for (int o = 0; o < (int)kPairSym; ++o) {
                const bool ok = (uint32_t)o < S;
                const uint32_t oc = ok ? (uint32_t)o : S - 1u;
                const float2 e0 = m.tab[((size_t)(blk * S + oc) * SM + 0) * 64 + lane];
                const float2 e1 = m.tab[((size_t)(blk * S + oc) * SM + 1) * 64 + lane];
                const uint32_t pb = lane ? blk : (blk ? blk - 1u : 0u), pl = lane ? lane - 1u : 63u;
                const bool pok = ok && (lane || blk);
                const float2 pe = m.tab[((size_t)(pb * S + oc) * SM + 1) * 64 + pl];
                const float val[3][2] = {{ok ? e0.x : kInf, ok ? e1.x : kInf}, {ok ? e0.y : kInf, ok ? e1.y : kInf},
                                         {pok ? pe.x : kInf, pok ? pe.y : kInf}};
#pragma unroll
                for (int k = 0; k < 3; ++k)
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int r = 2 * o + u;
                        if (r < 32) TA[k][r] = val[k][u];
                        else TB[k][r - 32] = val[k][u];
                    }
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) asm volatile("" : "+v"(TA[k]), "+v"(TB[k]));
        } else if constexpr (kT3) {
#pragma unroll
            for (int o = 0; o < (int)kPairSym; ++o) {
                const bool ok = (uint32_t)o < S;
                const uint32_t oc = ok ? (uint32_t)o : S - 1u;  // unconditional loads, then selects
                const float2 e0 = m.tab[((size_t)(blk * S + oc) * SM + 0) * 64 + lane];
                const float2 e1 = m.tab[((size_t)(blk * S + oc) * SM + 1) * 64 + lane];
                const float4 h = *reinterpret_cast<const float4*>(m.hc + oc * 8);
                // TM 3: {ea_0, ea_1}, {eb_0, eb_1}; otherwise {eb_0, ea_0}, {eb_1, ea_1}
                const float2 t1 = TM >= 3 ? make_float2(e0.y, e1.y) : e0, t2 = TM >= 3 ? make_float2(e0.x, e1.x) : e1;
                const float val[4][2] = {{ok ? t1.x : kInf, ok ? t1.y : kInf}, {ok ? t2.x : kInf, ok ? t2.y : kInf},
                                         {ok ? h.x : kInf, ok ? h.y : kInf}, {ok ? h.z : kInf, ok ? h.w : kInf}};
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int r = 2 * o + u;
                        if (r < 32) TA[k][r] = val[k][u];
                        else TB[k][r - 32] = val[k][u];
                    }
            }
            // opaque per-lane values: the heavy constants are wave-uniform, and the compiler would
            // otherwise keep them in SGPRs and copy them into the pinned registers at every step
#pragma unroll
            for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(TA[k]), "+v"(TB[k]));
        }
#ifdef SVH_PIPE_DIAG
        if (dbg) {  // stamp 13: the tables have arrived (a use of every table register)
#pragma unroll
            for (int k = 0; k < 4; ++k) asm volatile("" ::"v"(TA[k]), "v"(TB[k]));
            SVH_RT(13);
        }
#endif
        // heavy constants as lane tables (lane o: symbol o), extracted with v_readlane
        const bool lo = lane < S;
        const float cAS = lo ? m.hc[lane * 8 + 0] : kInf, cAF = lo ? m.hc[lane * 8 + 1] : kInf;
        const float cXSS = lo ? m.hc[lane * 8 + 2] : kInf, cXFF = lo ? m.hc[lane * 8 + 3] : kInf;
        const float cXSF = lo ? m.hc[lane * 8 + 4] : kInf;
        // ---- state at observation first-1
        if (beg == 0) {
            const uint32_t o0 = (uint32_t)uniform((int)sym[0]);
#pragma unroll
            for (int s = 0; s < SM; ++s) v[s] = m.e0[(size_t)o0 * P + p0 + s] + m.start[p0 + s];
            CF.y = m.rowF >= 0 ? ctab[o0 * 8 + 5] + m.startF : kInf;
            CF.x = (blk == 0 && lane == 0 && m.rowS >= 0) ? ctab[o0 * 8 + 6] + m.startS : kInf;
        } else {
            const float* vin = b.v_in + (size_t)b.v_in_row[q] * m.n;
#pragma unroll
            for (int s = 0; s < SM; ++s) {
                const uint32_t r = m.lrow[p0 + s];
                v[s] = r != kNoRow ? vin[r] : kInf;
            }
            CF.y = m.rowF >= 0 ? vin[m.rowF] : kInf;
            CF.x = (blk == 0 && lane == 0 && m.rowS >= 0) ? vin[m.rowS] : kInf;
        }

        // ---- decoded paths: outputs and the per-slot tie masks
        float* const pring_w = pring + w * 8 * kPQuadStride;
        // lane l's float4 in plane 0 of quad q (observations 4q, 4q+1 of the cycle of 32; plane 1,
        // kPPlane floats on, holds 4q+2, 4q+3)
        float* const pring_l = pring_w + lane * 4;
        float pst[8];  // this quad's {pm, c} pairs, written by two ds_write_b128 at its last step
        uint32_t* const cmq = PATHS ? b.cmask + b.cmask_off[q] : nullptr;
        float* const ckq = PATHS ? b.ckpt + b.ckpt_off[q] : nullptr;
        float2* const precq = PATHS ? b.prec + b.prec_off[q] : nullptr;
        float* const fckq = PATHS ? b.fck + b.fck_off[q] : nullptr;
        const uint32_t wstride = m.nblk * SM * 64;  // mask words per 32 rows
        auto store_masks = [&](uint32_t word, uint32_t rows) {  // rows 32*word .. +rows-1 are in macc
            if (kNoPStore) return;
#pragma unroll
            for (int s = 0; s < SM; ++s)
                cmq[(size_t)word * wstride + (blk * SM + s) * 64 + lane] = macc[s] << (32u - rows);
        };
        auto checkpoint = [&](uint32_t t) {  // t % kCkptEvery == 0: the light scores of t
            if (kNoPStore) return;
            float* d = ckq + (size_t)(t / kCkptEvery) * m.P + p0;
            if constexpr (SM == 2) {
                *reinterpret_cast<float2*>(d) = make_float2(v[0], v[1]);
            } else {
#pragma unroll
                for (int s = 0; s < SM; ++s) d[s] = v[s];
            }
        };
        // {light minimum of t-1, sink partial of t}: kept in registers for the 4 observations of a
        // quad and written by its last step as two ds_write_b128 (one LDS store per step cost 40 us
        // of the 388 us path kernel on the headline, profiles/r05_s11); single observations (head,
        // tail) write their own pair
        auto ring_put2 = [&](auto rc) {  // rc: the observation's place in its quad (compile time)
            constexpr uint32_t r = decltype(rc)::value;
            pst[2 * r] = last_pm;
            pst[2 * r + 1] = CF.x;
        };
        auto ring_flush = [&](uint32_t t) {  // t % 4 == 3: the quad of t is complete
            if (kNoPRing) {
                asm volatile("" ::"v"(pst[0]), "v"(pst[1]), "v"(pst[2]), "v"(pst[3]), "v"(pst[4]), "v"(pst[5]), "v"(pst[6]), "v"(pst[7]));
                return;
            }
            float* d = pring_l + ((t >> 2) & 7u) * kPQuadStride;
            *reinterpret_cast<float4*>(d) = make_float4(pst[0], pst[1], pst[2], pst[3]);
            *reinterpret_cast<float4*>(d + kPPlane) = make_float4(pst[4], pst[5], pst[6], pst[7]);
        };
        auto ring_put1 = [&](uint32_t t) {
            *reinterpret_cast<float2*>(pring_l + ((t >> 2) & 7u) * kPQuadStride + ((t & 3u) >> 1) * kPPlane + (t & 1u) * 2) =
                make_float2(last_pm, CF.x);
        };
        // fold observations tb .. tb+31 (tb % 32 == 0) and store those in [1, thi): lane l takes
        // observation o = l % 32 over the half-wave of source lanes l / 32, then the two halves
        // combine (one swizzle) and lanes 0..31 store one record per observation
        auto reduce_ring = [&](uint32_t tb, uint32_t thi) {
            if (kNoFold || kNoPRing) return;
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const uint32_t o = lane & 31u, H = lane >> 5;
            const float* rp = pring_w + (o >> 2) * kPQuadStride + ((o & 3u) >> 1) * kPPlane + H * (32 * 4) + (o & 1u) * 2;
            float mm = kInf, cc = kInf;
#pragma unroll
            for (int L = 0; L < 32; ++L) {
                const float2 e = *reinterpret_cast<const float2*>(rp + L * 4);
                mm = fminf(mm, e.x);
                cc = fminf(cc, e.y);
            }
            mm = fminf(mm, __shfl_xor(mm, 32));
            cc = fminf(cc, __shfl_xor(cc, 32));
            const uint32_t tt = tb + o;
            if (kNoPStore) {
                asm volatile("" ::"v"(mm), "v"(cc));  // the fold still runs
                return;
            }
            if (H == 0 && tt >= 1 && tt < thi) precq[(size_t)blk * len + tt] = make_float2(mm, cc);
        };
        // after the step of observation t (compile-time positions in the unrolled body)
        auto paths_after = [&](uint32_t t, auto maskc, auto ckc, auto redc, auto rc) {
            if constexpr (PATHS) {
                ring_put2(rc);
                if constexpr (decltype(rc)::value == 3) ring_flush(t);
                if constexpr (decltype(maskc)::value) {
                    if (t >= 32) store_masks((t >> 5) - 1, 32);
                    if (blk == 0 && lane == 0) fckq[t >> 5] = CF.y;
                }
                if constexpr (decltype(ckc)::value) checkpoint(t);
                if constexpr (decltype(redc)::value) reduce_ring(t - 31, len);
            }
        };
        auto paths_after_rt = [&](uint32_t t) {  // runtime positions (head / tail)
            if constexpr (PATHS) {
                ring_put1(t);
                if ((t & 31u) == 0) {
                    if (t >= 32) store_masks((t >> 5) - 1, 32);
                    if (blk == 0 && lane == 0) fckq[t >> 5] = CF.y;
                }
                if ((t & (kCkptEvery - 1)) == 0) checkpoint(t);
                if ((t & 31u) == 31u) reduce_ring(t - 31, len);
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
        // Observations run in groups of 32 aligned to `first` (tb = first % 32; 0 for the path
        // variants, whose records sit at absolute multiples of 32): the body starts at first
        // itself, with no head of single observations (each one an LDS or L2 round trip, and the
        // head's cost adds up along the chain of waves).  What is indexed by the position in the
        // cycle of 32 -- symbol windows, LDS ring slots -- uses u = t - tb; counts, granules and
        // tags use t.
#ifdef SVH_PIPE_HEAD  // A/B diagnostic: the head of single observations of before
        const uint32_t tb = 0u;
#else
        const uint32_t tb = PATHS ? 0u : (first & 31u);
#endif
        auto load_window_raw = [&](uint32_t wi) -> uint4 {  // lane l: symbols of u = 1024 wi + 16 l ..
            const uint32_t off = wi * kPipeWindow + lane * 16 + tb;
            if ((tb & 15u) == 0)
                return off < slen ? *reinterpret_cast<const uint4*>(sym + off) : make_uint4(0, 0, 0, 0);
            // unaligned: two aligned 16-byte loads and a byte funnel shift (once per window)
            const uint32_t a = off & ~15u, ws = (tb & 15u) >> 2, bs = tb & 3u;
            const uint4 c0 = a < slen ? *reinterpret_cast<const uint4*>(sym + a) : make_uint4(0, 0, 0, 0);
            const uint4 c1 = a + 16 < slen ? *reinterpret_cast<const uint4*>(sym + a + 16) : make_uint4(0, 0, 0, 0);
            auto pick = [&](uint32_t i) -> uint32_t {  // word ws + i of c0 | c1 (selects, no scratch)
                const uint32_t k = ws + i;
                uint32_t r = c0.x;
                r = k == 1 ? c0.y : r;
                r = k == 2 ? c0.z : r;
                r = k == 3 ? c0.w : r;
                r = k == 4 ? c1.x : r;
                r = k == 5 ? c1.y : r;
                r = k == 6 ? c1.z : r;
                r = k == 7 ? c1.w : r;
                return r;
            };
            const uint32_t p0 = pick(0), p1 = pick(1), p2 = pick(2), p3 = pick(3), p4 = pick(4);
            return make_uint4(__builtin_amdgcn_alignbyte(p1, p0, bs), __builtin_amdgcn_alignbyte(p2, p1, bs),
                              __builtin_amdgcn_alignbyte(p3, p2, bs), __builtin_amdgcn_alignbyte(p4, p3, bs));
        };
        auto load_window = [&](uint32_t wi) -> uint4 {  // mode 3: every symbol byte doubled (2o < 64)
            const uint4 w4 = load_window_raw(wi);
            if constexpr (kT3) return make_uint4(w4.x << 1, w4.y << 1, w4.z << 1, w4.w << 1);
            return w4;
        };
        uint32_t cwi = (first - tb) >> 10;
        uint4 cw = load_window(cwi), nw = load_window(cwi + 1);
        // The wait budget is per window: a new window resets a healthy counter (a give-up sticks),
        // so no sequence length exhausts it while a stuck wait still gives up within one budget.
        auto window_for = [&](uint32_t t) {  // uniform; windows advance one at a time
            if (((t - tb) >> 10) != cwi) {
                cw = nw;
                ++cwi;
                nw = load_window(cwi + 1);
                spins = spins > kSpinLimit ? spins : 0u;
            }
        };
        auto sym1 = [&](uint32_t t) -> uint32_t {  // symbol of observation t (slow path)
            const uint32_t r = (t - tb) & 1023u, ln = r >> 4, d = (r >> 2) & 3u;
            const uint32_t wd = d == 0 ? readlane_u(cw.x, ln) : d == 1 ? readlane_u(cw.y, ln)
                              : d == 2 ? readlane_u(cw.z, ln) : readlane_u(cw.w, ln);
            return (wd >> ((r & 3u) * 8)) & 0xFFu;
        };

        // ---- one observation with symbol o; bnd = the previous block's last score at t-1
        // `in`: ChainIn<R>, slot 0's chain input (see ChainIn)
        auto step = [&](uint32_t o, auto in) {
            constexpr int R = decltype(in)::value;
            float xa[SM], xb[SM];  // feeder and chain terms of every slot
            if constexpr (TM == 2 || TM == 4) {  // o is 2 x the symbol: the table reads are indexed operands
                // of the adds that use them (one gpr_idx(SRC0) block; only eb_0 is moved out, for
                // slot 0's DPP chain add)
                const float pm = fminf(v[0], v[1]);  // the heavy side reads the scores of t-1
                f2 pmv;  // the packed add reads the low half twice (op_sel_hi): the high half is never read
                pmv.x = pm;
                float eb0;
                f2 s1, s2;  // {A_S + m, A_F + m}, {X_SS + c, X_FF + F}
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#pragma clang diagnostic ignored "-Wuninitialized"
                if constexpr (TM == 2) {
                asm("s_set_gpr_idx_on %[o], gpr_idx(SRC0)\n\t"
                    "v_mov_b32 %[eb0], v2\n\t"
                    "v_add_f32 %[xa0], v3, %[f]\n\t"
                    "v_add_f32 %[xa1], v43, %[f]\n\t"
                    "v_add_f32 %[xb1], v42, %[v0]\n\t"
                    "v_pk_add_f32 %[s1], v[82:83], %[pm] op_sel_hi:[1,0]\n\t"
                    "v_pk_add_f32 %[s2], v[122:123], %[cf]\n\t"
                    "s_set_gpr_idx_off"
                    : [eb0] "=&v"(eb0), [xa0] "=&v"(xa[0]), [xa1] "=&v"(xa[1]), [xb1] "=&v"(xb[1]), [s1] "=&v"(s1),
                      [s2] "=&v"(s2)
                    : [o] "s"(o), [f] "v"(CF.y), [v0] "v"(v[0]), [pm] "v"(pmv), [cf] "v"(CF), "{v[2:33]}"(TA[0]),
                      "{v[34:41]}"(TB[0]), "{v[42:73]}"(TA[1]), "{v[74:81]}"(TB[1]), "{v[82:113]}"(TA[2]),
                      "{v[114:121]}"(TB[2]), "{v[122:153]}"(TA[3]), "{v[154:161]}"(TB[3])
                    : "m0");
                } else {  // T1 = {ea_0, ea_1}: one packed feeder add, F from the high half of CF
                f2 xap;
                asm("s_set_gpr_idx_on %[o], gpr_idx(SRC0)\n\t"
                    "v_mov_b32 %[eb0], v42\n\t"
                    "v_pk_add_f32 %[xa], v[2:3], %[cf] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
                    "v_add_f32 %[xb1], v43, %[v0]\n\t"
                    "v_pk_add_f32 %[s1], v[82:83], %[pm] op_sel_hi:[1,0]\n\t"
                    "v_pk_add_f32 %[s2], v[122:123], %[cf]\n\t"
                    "s_set_gpr_idx_off"
                    : [eb0] "=&v"(eb0), [xa] "=&v"(xap), [xb1] "=&v"(xb[1]), [s1] "=&v"(s1), [s2] "=&v"(s2)
                    : [o] "s"(o), [v0] "v"(v[0]), [pm] "v"(pmv), [cf] "v"(CF), "{v[2:33]}"(TA[0]),
                      "{v[34:41]}"(TB[0]), "{v[42:73]}"(TA[1]), "{v[74:81]}"(TB[1]), "{v[82:113]}"(TA[2]),
                      "{v[114:121]}"(TB[2]), "{v[122:153]}"(TA[3]), "{v[154:161]}"(TB[3])
                    : "m0");
                xa[0] = xap.x;
                xa[1] = xap.y;
                }
#pragma clang diagnostic pop
                xb[0] = chain_b<R>(eb0, in.b, v[1]);
                float cn = fminf(s1.x, s2.x);
                if constexpr (SX) cn = fminf(cn, readlane_f(cXSF, o >> 1) + CF.y);
                asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, 0, %0, vcc"
                             : "+v"(viol)
                             : "v"(s1.y), "v"(s2.y)
                             : "vcc");
                auto push = [&](int s, float a, float bb) {
                    if constexpr (PATHS == 2) push_le(macc[s], a, bb);
                    else if constexpr (PATHS == 1) push_lt_eqc(macc[s], a, bb, pmC[s]);
                };
                if constexpr (PATHS) last_pm = pm;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    if constexpr (PATHS) push(s, xa[s], xb[s]);
                    v[s] = fminf(xa[s], xb[s]);
                }
                CF = (f2){cn, s2.y};
                return;
            } else if constexpr (kT4) {  // o is 2 x the symbol: four 64-bit moves out of the pair tables
                f2 p0, p1, kS, kX;  // {eb_0, ea_0}, {eb_1, ea_1}, {A_S, A_F}, {X_SS, X_FF}
                // M0 is reserved (clang warns on the clobber); the kernel uses it nowhere else
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
                asm("s_set_gpr_idx_on %[o], gpr_idx(SRC0)\n\t"
                    "v_mov_b64 %[p0], v[2:3]\n\t"
                    "v_mov_b64 %[p1], v[42:43]\n\t"
                    "v_mov_b64 %[ks], v[82:83]\n\t"
                    "v_mov_b64 %[kx], v[122:123]\n\t"
                    "s_set_gpr_idx_off"
                    : [p0] "=&v"(p0), [p1] "=&v"(p1), [ks] "=&v"(kS), [kx] "=&v"(kX)
                    : [o] "s"(o), "{v[2:33]}"(TA[0]), "{v[34:41]}"(TB[0]), "{v[42:73]}"(TA[1]), "{v[74:81]}"(TB[1]),
                      "{v[82:113]}"(TA[2]), "{v[114:121]}"(TB[2]), "{v[122:153]}"(TA[3]), "{v[154:161]}"(TB[3])
                    : "m0");
#pragma clang diagnostic pop
                if constexpr (TM == 3) {  // p0 = {ea_0, ea_1}, p1 = {eb_0, eb_1}
                    f2 xap;
                    chain_terms_pk<R>(xb[0], xap, p0, p1.x, in.b, CF, v[1]);
                    xa[0] = xap.x;
                    xa[1] = xap.y;
                    xb[1] = p1.y + v[0];
                } else {
                    if constexpr (R < 0) chain_terms(xb[0], xa[0], p0.x, p0.y, in.b, CF.y, v[1]);
                    else chain_terms_v<R>(xb[0], xa[0], p0.x, p0.y, in.b, CF.y, v[1]);
                    xa[1] = p1.y + CF.y;
                    xb[1] = p1.x + v[0];
                }
                const float pm = fminf(v[0], v[1]);
                const f2 s1 = kS + (f2){pm, pm};  // A_S + m, A_F + m
                const f2 s2 = kX + CF;            // X_SS + c, X_FF + F
                float cn = fminf(s1.x, s2.x);
                if constexpr (SX) cn = fminf(cn, readlane_f(cXSF, o >> 1) + CF.y);
                asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, 0, %0, vcc"
                             : "+v"(viol)
                             : "v"(s1.y), "v"(s2.y)
                             : "vcc");
                auto push = [&](int s, float a, float bb) {
                    if constexpr (PATHS == 2) push_le(macc[s], a, bb);
                    else if constexpr (PATHS == 1) push_lt_eqc(macc[s], a, bb, pmC[s]);
                };
                if constexpr (PATHS) last_pm = pm;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    if constexpr (PATHS) push(s, xa[s], xb[s]);
                    v[s] = fminf(xa[s], xb[s]);
                }
                CF = (f2){cn, s2.y};
                return;
            }
            const float kas = readlane_f(cAS, o), kaf = readlane_f(cAF, o);
            const float kxss = readlane_f(cXSS, o), kxff = readlane_f(cXFF, o);
            {
                float eb[SM], ea[SM];
#pragma unroll
                for (int s = 0; s < SM; ++s) {
                    eb[s] = EB[s][o];
                    ea[s] = EA[s][o];
                }
#pragma unroll
                for (int s = 0; s < SM; ++s) asm volatile("" : "+v"(eb[s]), "+v"(ea[s]));  // one idx block
                if constexpr (R < 0) chain_terms(xb[0], xa[0], eb[0], ea[0], in.b, CF.y, v[SM - 1]);
                else chain_terms_v<R>(xb[0], xa[0], eb[0], ea[0], in.b, CF.y, v[SM - 1]);
#pragma unroll
                for (int s = 1; s < SM; ++s) {
                    xa[s] = ea[s] + CF.y;
                    xb[s] = eb[s] + v[s - 1];
                }
            }
            float vn[SM];
            auto push = [&](int s, float a, float bb) {  // PATHS: F's term taken (row t-1's bit)
                if constexpr (PATHS == 2) push_le(macc[s], a, bb);
                else if constexpr (PATHS == 1) push_lt_eqc(macc[s], a, bb, pmC[s]);
            };
#pragma unroll
            for (int s = 0; s < SM; ++s) {
                vn[s] = fminf(xa[s], xb[s]);
                if constexpr (PATHS) push(s, xa[s], xb[s]);
            }
            // heavy side from the scores of t-1
            float pm = v[0];
#pragma unroll
            for (int s = 1; s < SM; ++s) pm = fminf(pm, v[s]);
            if constexpr (PATHS) last_pm = pm;
            const f2 s1 = (f2){kas, kaf} + (f2){pm, pm};  // A_S + m, A_F + m
            const f2 s2 = (f2){kxss, kxff} + CF;          // X_SS + c, X_FF + F
            float cn = fminf(s1.x, s2.x);
            if constexpr (SX) cn = fminf(cn, readlane_f(cXSF, o) + CF.y);
            // viol += [A_F + m < F'] per lane: compare into VCC, add with carry-in (two VALU, no
            // VALU -> SALU dependency per step)
            asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, 0, %0, vcc"
                         : "+v"(viol)
                         : "v"(s1.y), "v"(s2.y)
                         : "vcc");
            CF = (f2){cn, s2.y};
#pragma unroll
            for (int s = 0; s < SM; ++s) v[s] = vn[s];
        };

        // ---- L2: one chunk of _spec level 2 (observations t - 1, t with symbols s1, s2; o1, o2 = 2 x
        // the symbols).  GraphBLAS_spec_impl.cpp:15-36, 66-81: v'[j] = min_m fl(H[j][m] + v[m]) with
        // H[j][m] = min_p fl(M_s2[j][p] + M_s1[p][m]), M_s[j][p] = fl(E_s[j] + T^T[j][p]); fl(x + v) is
        // monotone in x, so bit for bit v'[j] = min over the two-hop paths j <- p <- m of
        // fl(fl(M_s2[j][p] + M_s1[p][m]) + v[m]) (spec2.hip (1)).  In the chain shape the paths into a
        // light position j are (j-1, j-2), (j-1, F), (F, F) and (F, light m); into F: (F, F), (F, m),
        // (q, q-1), (q, F) for every light q; into S: (S, S), (S, m), (q, q-1), (q, F) [+ (S, F),
        // (F, F), (F, m) with SX].  So, with eb/ea the folded tables of level 0:
        //   v'_j = min(fl(fl(eb_j(s2) + eb_{j-1}(s1)) + v_{j-2}),
        //              fl(min(fl(eb_j(s2) + ea_{j-1}(s1)), fl(ea_j(s2) + X_FF(s1))) + F))     [exact]
        //          and the (F, m) term fl(fl(ea_j(s2) + A_F(s1)) + mu), which is speculated never to win;
        //   F' = fl(fl(X_FF(s2) + X_FF(s1)) + F), speculated: every other term of F checked >= F' exactly
        //        in the lane that holds it ((F, m) with the lane's own minimum: fl(a + .) is monotone);
        //   S: every term evaluated in the lane that holds it, S = min over lanes (as at level 0).
        // The two light positions two apart form independent chains (even and odd), each depending on
        // position j - 2 of the previous chunk: lane - 1's same slot, the previous block's last two
        // scores for lane 0.  The speculated (F, m) term of position j is bounded without mu: with all
        // scores >= 0 (the host's check) each fl() is within (1 +- u) of the exact sum, so
        // fl(fl(e + A_F) + mu) >= fl(fl(e + X_FF) + F) for every e in [0, emax2] once
        // fl(A_F + mu_lane) >= fl(R + fl(emax2 + R) 2^-20), R = fl(X_FF + F): the margin 16u (emax2 + R)
        // exceeds the 4u (e + X_FF + F) the four roundings can close (derivation in DESIGN.md 5j).
        // The lane holding mu passes it whenever any lane does not fail, so a row with no failing lane
        // never takes the (F, m) term.  Failing rows are flagged (viol) and re-run by spec2_kernel.
        auto step2 = [&](uint32_t o1, uint32_t o2, float vp0, float vp1) {
            if constexpr (L2) {
                f2 e1, a1, pr, e2, a2;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
                asm("s_set_gpr_idx_on %[o], gpr_idx(SRC0)\n\t"
                    "v_mov_b64 %[e], v[2:3]\n\t"
                    "v_mov_b64 %[a], v[42:43]\n\t"
                    "v_mov_b64 %[p], v[82:83]\n\t"
                    "s_set_gpr_idx_off"
                    : [e] "=&v"(e1), [a] "=&v"(a1), [p] "=&v"(pr)
                    : [o] "s"(o1), "{v[2:33]}"(TA[0]), "{v[34:41]}"(TB[0]), "{v[42:73]}"(TA[1]), "{v[74:81]}"(TB[1]),
                      "{v[82:113]}"(TA[2]), "{v[114:121]}"(TB[2])
                    : "m0");
                asm("s_set_gpr_idx_on %[o], gpr_idx(SRC0)\n\t"
                    "v_mov_b64 %[e], v[2:3]\n\t"
                    "v_mov_b64 %[a], v[42:43]\n\t"
                    "s_set_gpr_idx_off"
                    : [e] "=&v"(e2), [a] "=&v"(a2)
                    : [o] "s"(o2), "{v[2:33]}"(TA[0]), "{v[34:41]}"(TB[0]), "{v[42:73]}"(TA[1]), "{v[74:81]}"(TB[1]),
                      "{v[82:113]}"(TA[2]), "{v[114:121]}"(TB[2])
                    : "m0");
#pragma clang diagnostic pop
                // heavy constants {A_S, A_F}, {X_SS, X_FF}, {X_SF} of s1 and s2 from the lane tables
                const uint32_t u1 = o1 >> 1, u2 = o2 >> 1;
                const f2 h1 = {readlane_f(cAS, u1), readlane_f(cAF, u1)}, x1 = {readlane_f(cXSS, u1), readlane_f(cXFF, u1)};
                const f2 h2 = {readlane_f(cAS, u2), readlane_f(cAF, u2)}, x2 = {readlane_f(cXSS, u2), readlane_f(cXFF, u2)};
                f2 s1 = {kInf, kInf}, s2 = {kInf, kInf};
                if constexpr (SX) {
                    s1.x = readlane_f(cXSF, u1);
                    s2.x = readlane_f(cXSF, u2);
                }
                const float F = CF.y, c = CF.x;
                const float pm = fminf(v[0], v[1]);  // the lane's minimum of the scores before the chunk
                // light positions (slot 0: j - 1 is p0 - 1, the pred table; slot 1: j - 1 is slot 0)
                const f2 cb = e2 + (f2){pr.x, e1.x};                  // fl(eb_j(s2) + eb_{j-1}(s1))
                const f2 f1 = e2 + (f2){pr.y, a1.x};                  // fl(eb_j(s2) + ea_{j-1}(s1))
                const f2 fx = a2 + (f2){x1.y, x1.y};                  // fl(ea_j(s2) + X_FF(s1))
                const f2 fa = (f2){fminf(f1.x, fx.x), fminf(f1.y, fx.y)};
                const f2 xa = fa + (f2){F, F};
                const f2 xb = cb + (f2){vp0, vp1};
                // F: the speculated (F, F) term and every other term of F's row
                const float Fn = (x2.y + x1.y) + F;
                const f2 qb = ((f2){h2.y, h2.y} + (f2){e1.x, e1.y}) + (f2){vp1, v[0]};  // (q, q-1): v_{q-1}
                const f2 qa = ((f2){h2.y, h2.y} + a1) + (f2){F, F};                     // (q, F)
                float nm = (x2.y + h1.y) + pm;                                          // (F, m)
                nm = fminf(nm, fminf(fminf(qb.x, qb.y), fminf(qa.x, qa.y)));
                // the margin bound of the light positions' (F, m) term
                const float Rf = x1.y + F;
                const float thr = Rf + (m.emax2 + Rf) * 0x1p-20f;
                const float Lf = h1.y + pm;
                asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, 0, %0, vcc"
                             : "+v"(viol)
                             : "v"(nm), "v"(Fn)
                             : "vcc");
                asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, 0, %0, vcc"
                             : "+v"(viol)
                             : "v"(Lf), "v"(thr)
                             : "vcc");
                // S (this lane's partial)
                const f2 sb = ((f2){h2.x, h2.x} + (f2){e1.x, e1.y}) + (f2){vp1, v[0]};  // (q, q-1)
                const f2 sa = ((f2){h2.x, h2.x} + a1) + (f2){F, F};                     // (q, F)
                float cn = fminf((x2.x + x1.x) + c, (x2.x + h1.x) + pm);               // (S, S), (S, m)
                cn = fminf(cn, fminf(fminf(sb.x, sb.y), fminf(sa.x, sa.y)));
                if constexpr (SX) {
                    cn = fminf(cn, (x2.x + s1.x) + F);   // (S, F)
                    cn = fminf(cn, (s2.x + x1.y) + F);   // (F, F)
                    cn = fminf(cn, (s2.x + h1.y) + pm);  // (F, m)
                }
                v[0] = fminf(xa.x, xb.x);
                v[1] = fminf(xa.y, xb.y);
                CF = (f2){cn, Fn};
            }
        };

        // ---- exchange state
        float* const ring_w = ring + w * kR * 64;
        const float* const ring_prev = ring_w - kR * 64;
        uint32_t* const cnt_w = cnt + w;
        const uint32_t cnt_addr = lds_addr(cnt_w);
        auto put_cnt = [&](uint32_t val) { lds_put1(cnt_addr, val); };
        uint64_t* const gin = x.gran + ((size_t)q * (G - 1) + (g - 1)) * kGR;  // src == 2
        uint64_t* const gout = x.gran + ((size_t)q * (G - 1) + g) * kGR;       // dst == 2
        uint64_t* const cons_in = reinterpret_cast<uint64_t*>(x.cons) + (size_t)q * G + g;      // src == 2 publishes
        const uint64_t* const cons_out = reinterpret_cast<const uint64_t*>(x.cons) + (size_t)q * G + g + 1;  // dst == 2 reads
        // SVH_PIPE_XHELP: wave 1 publishes this workgroup's progress (helped: wave 0 does not), wave
        // W - 2 forwards the consumer's word to wave W - 1 through consf (cnt[14..15])
        constexpr bool kXh = SVH_PIPE_XHELP && W >= 3;
        static_assert(W <= 14, "cnt[14..15] holds the forwarded progress word");
        uint64_t* const consf = reinterpret_cast<uint64_t*>(cnt + 14);
        const bool helped = kXh && g > 0 && g * W + 1 < m.nblk;
        const bool hpub = helped && w == 1;
        const bool hrd = kXh && w == (uint32_t)W - 2 && (g + 1) * W < m.nblk;
        float bprev = kInf;  // boundary score of observation t-1 for the next step (uniform)
    float bprev2 = kInf;  // L2: ... of t-2 (a chunk's step reads the previous block's two last scores)

        auto give_up = [&]() -> bool { return ++spins > kSpinLimit; };
        // SVH_PIPE_XL: is workgroup og of this row on this wave's XCD?  (bounded poll of its id; not
        // known in time: no, i.e. write-through stores, always correct)
        auto xcc_local = [&](uint32_t og) -> bool {
#if SVH_PIPE_XL
            if (!x.xcc) return false;
            const uint32_t* p = x.xcc + (size_t)q * G + og;
            for (int i = 0; i < 32; ++i) {
                const uint32_t wv = (uint32_t)uniform((int)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if ((wv >> 4) == (ep & 0x0FFFFFFFu)) return (wv & 0xFu) == my_xcc;
                __builtin_amdgcn_s_sleep(4);
            }
#endif
            (void)og;
            return false;
        };
        bool gran_plain = false, cons_plain = false;
        // granule / progress-word stores: plain when the reader shares this XCD (SVH_PIPE_XL)
        // (a plain store is a relaxed atomic store at wavefront scope: the same unflagged
        // global_store as `*a = v64`, but one the compiler may not tear, merge or sink)
        auto st_gran = [&](uint64_t* a, uint64_t v64) {
            if (SVH_PIPE_XL && gran_plain) __hip_atomic_store(a, v64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            else g_st64(a, v64);
        };
        auto st_cons = [&](uint64_t v64) {
            if (SVH_PIPE_XL && cons_plain) __hip_atomic_store(cons_in, v64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            else g_st64(cons_in, v64);
        };
        // wait until the previous wave has published observations < need
        auto wait_prev = [&](uint32_t need) {
            if (kNoWait) return;
            while ((uint32_t)uniform((int)lds_ld32_slow(cnt_w - 1)) < need) {
                if (dbg) ++dg[3];
                if (give_up()) break;
                __builtin_amdgcn_s_sleep(1);
            }
        };
        // flow control: the next wave has consumed observations < need
        auto wait_next = [&](uint32_t need) {
            if (kNoWait) return;
            while ((int)uniform((int)lds_ld32_slow(cnt_w + 1)) < (int)need) {
                if (dbg) ++dg[4];
                if (give_up()) break;
                __builtin_amdgcn_s_sleep(1);
            }
        };
        // The boundary score of observation s from the previous workgroup's granules (uniform), for
        // the single observations (the tail, the path variants' head): eight granules per poll
        // (lanes 0..7: s .. s+7), one L2 round trip per 8 observations instead of one each.
        // Only granules this wave reads (observations <= len-2) are awaited.
        float gvec = 0.0f;
        uint32_t gbase = 0x80000000u;  // no observation index reaches it: the first call loads
        auto gran_single = [&](uint32_t s) -> float {
            if (s - gbase >= 8u) {
                gbase = s;
                const uint32_t sl = s + (lane & 7u);
                const bool need = lane < 8u && sl + 1u < len;
                const uint64_t* p = gin + (sl & (kGR - 1));
                uint64_t gv = g_ld64(p);
                while (!kNoWait && __builtin_amdgcn_ballot_w64(need && (uint32_t)(gv >> 32) != gtag(ep, sl)) != 0) {
                    if (dbg) ++dg[5];
                    if (give_up()) break;
                    __builtin_amdgcn_s_sleep(1);
                    gv = g_ld64(p);
                }
                gvec = __builtin_bit_cast(float, (uint32_t)gv);
            }
            return readlane_f(gvec, s - gbase);
        };
        auto cons_ok = [&](uint64_t c, uint32_t need) -> bool {  // consumer progress word vs need
            return (uint32_t)(c >> 32) == ep && (int)(uint32_t)c >= (int)need;
        };
        auto uni64 = [](uint64_t c) -> uint64_t {
            return (uint64_t)(uint32_t)uniform((int)(uint32_t)c) | ((uint64_t)(uint32_t)uniform((int)(uint32_t)(c >> 32)) << 32);
        };
        auto wait_cons = [&](uint32_t need) {
            if (kNoWait) return;
            uint64_t c = g_ld64_slow(cons_out);
            while (!cons_ok(uni64(c), need)) {
                if (dbg) ++dg[6];
                if (give_up()) break;
                __builtin_amdgcn_s_sleep(2);
                c = g_ld64_slow(cons_out);
            }
        };
        auto put_gran1 = [&](uint32_t s, float val) {  // single observation (slow path), lane 0 stores
            const uint64_t gv = ((uint64_t)gtag(ep, s) << 32) | __builtin_bit_cast(uint32_t, val);
            if (lane == 0) g_st64(gout + (s & (kGR - 1)), gv);
        };
        auto ring_put = [&](uint32_t t, float val) { ring_w[ring_idx((t - tb) & (kR - 1), lane)] = val; };

        // The sweep, with the boundary roles as compile-time constants (one code path per role).
        auto sweep = [&](auto srcc, auto dstc) {
            constexpr uint32_t GPF = kGpf;  // granule groups in flight (SRC 2)
            // The granule prefetch is an asm load into a loop-carried register (g_prefetch64) where
            // the register budget leaves the compiler no reason to move it; the level-2 body runs at
            // the 256-VGPR limit and copied the pending register to an AGPR before the load landed
            // (a stale granule then passed the lap tag, and the late return can overwrite a
            // re-used register), so there the prefetch is a load the compiler tracks.
            // tools/check_prefetch.py rejects a build whose asm prefetch is read before its wait.
            constexpr bool kPfAsm = !L2;
            auto prefetch = [&](uint64_t& d, const uint64_t* p) {
                if constexpr (kPfAsm) g_prefetch64(d, p);
                else d = g_ld64(p);
            };
            constexpr int SRC = decltype(srcc)::value, DST = decltype(dstc)::value;
            // one observation outside the unrolled groups: per-observation waits
            auto single = [&](uint32_t t) {
                window_for(t);
                const uint32_t o = (uint32_t)uniform((int)sym1(t));
                if constexpr (DST == 1) wait_next((int)t - (int)kR + 1);
                if constexpr (DST == 2) {
                    if ((t & 63u) == 0) wait_cons((int)t - (int)kGR + 64);
                }
                if constexpr (L2) {
                    // t odd: the chunk's first observation (nothing to compute; publish v_1 of the
                    // state before it); t even: the chunk (publish v_0 of the state after it)
                    if ((t & 1u) == 0) step2(sym1(t - 1), o, shr_in<0>(v[0], bprev2), shr_in<0>(v[1], bprev));
                    const float pub = (t & 1u) ? v[1] : v[0];
                    ring_put(t, pub);
                    if constexpr (DST == 2) put_gran1(t, readlane_f(pub, 63));
                } else {
                    step(o, ChainIn<-1>{bprev});
                    ring_put(t, v[SM - 1]);
                    if constexpr (DST == 2) put_gran1(t, readlane_f(v[SM - 1], 63));
                }
                paths_after_rt(t);
                if (t + 1 < len) {  // fetch the boundary score of t for the next step
                    bprev2 = bprev;
                    if constexpr (SRC == 1) {
                        wait_prev(t + 1);
                        asm volatile("" ::: "memory");
                        bprev = readlane_f(ring_prev[ring_idx((t - tb) & (kR - 1), 63)], 0);
                    } else if constexpr (SRC == 2) {
                        bprev = gran_single(t);
                    }
                }
                asm volatile("" ::: "memory");
                put_cnt(t + 1);
                if ((SRC == 2 && !helped) || (SRC == 1 && hpub)) {
                    if (lane == 0) g_st64(cons_in, ((uint64_t)ep << 32) | (t + 1));
                }
            };

            if constexpr (SVH_PIPE_XL && DST == 2) gran_plain = xcc_local(g + 1);
            if constexpr (SVH_PIPE_XL && SRC == 2) cons_plain = xcc_local(g - 1);
            if constexpr (SVH_PIPE_XL && SRC == 1 && kXh) {
                if (hpub) cons_plain = xcc_local(g - 1);
            }
            // publish the state at first-1 and fetch the boundary of first-1 (L2: first - 1 = 0 is
            // even, the published score is v_0)
            ring_put(first - 1, v[L2 ? 0 : SM - 1]);
            if constexpr (DST == 2) put_gran1(first - 1, readlane_f(v[L2 ? 0 : SM - 1], 63));
            asm volatile("" ::: "memory");
            put_cnt(first);
            // initial progress (observations < first are done), published before the first wait:
            // a row that starts mid-sequence at a multiple of 64 would otherwise leave its producer's
            // first flow-control wait on a stale word while wave 0 waits for that producer's
            // granules (the poll awaits observations up to first+6)
            if ((SRC == 2 && !helped) || (SRC == 1 && hpub)) {
                if (lane == 0) g_st64(cons_in, ((uint64_t)ep << 32) | first);
            }
            if constexpr (SRC == 1) {
                wait_prev(first);
                asm volatile("" ::: "memory");
                bprev = readlane_f(ring_prev[ring_idx((first - 1 - tb) & (kR - 1), 63)], 0);
            } else if constexpr (SRC == 2) {
                bprev = gran_single(first - 1);
            }

            uint32_t t = first;
            unsigned long long c0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
            SVH_RT(9);
            // head: single observations up to the first group of 32 (none unless tb is forced to 0)
            for (; t < len && ((t - tb) & 31u); ++t) single(t);
            if (dbg) {
                const unsigned long long c1 = __builtin_amdgcn_s_memtime();
                dg[1] = c1 - c0;
                c0 = c1;
            }

            // body: 32 observations per iteration, four groups of 8
            if (t + 32 <= len) {
                uint64_t gq[GPF] = {};  // SRC 2: granule groups in flight
                if constexpr (SRC == 2) {
#pragma unroll
                    for (uint32_t j = 0; j < GPF; ++j) prefetch(gq[j], gin + ((t + 8 * j + (lane & 7u)) & (kGR - 1)));
                }
                float gpend = 0.0f;    // DST 2: the previous group's boundary scores (lanes 0..7),
                uint32_t gpend_t = 0;  // read back from the ring one group before they are stored
                uint64_t cons_v = 0;   // DST 2: prefetched progress word of the consumer
                if constexpr (DST == 2) cons_v = g_ld64(cons_out);
                uint64_t cons_h = 0;   // SVH_PIPE_XHELP, wave W - 2: the word loaded for consf
                if constexpr (DST == 1 && kXh) {
                    if (hrd) cons_h = g_ld64(cons_out);
                }
                // counts of the neighbouring waves, read two observations before the end of a group
                uint32_t pc_rd = 0, nc_rd = 0;
                if constexpr (DST == 1) nc_rd = lds_ld32(cnt_w + 1);
                // boundary vectors (lanes 0..7 = the previous block's last scores of a group's 8
                // observations): the previous group's (lane 7 feeds the first step) and, SRC 1,
                // the next group's, read one group ahead whenever the producer is far enough
                float bv_prev = bprev;  // lane 7 (all lanes) = boundary of t-1
                // SRC 1: the next group's vector, loaded at the end of every group (stale unless
                // next_ok) into this one loop-carried register, re-loaded there when it was stale
                float bv_next = kInf;
                float bv_spec = kInf;  // SVH_PIPE_EARLYV: the next group's vector read at step 4
                bool next_ok = false;
                if constexpr (SRC == 1) bv_next = ring_prev[ring_idx(lane & 7u, 63)];  // group at t (u % 32 == 0)
                while (t + 32 <= len) {
                  // the window of t, loaded and waited for here (an asm use), so no load of it is
                  // pending inside the iterations: the compiler would otherwise wait for every
                  // vector-memory operation (granule prefetches and stores included) before each
                  // iteration's reads of the window
                  cwi = (t - tb) >> 10;
                  cw = load_window(cwi);
                  asm volatile("" ::"v"(cw.x), "v"(cw.y), "v"(cw.z), "v"(cw.w));
                  spins = spins > kSpinLimit ? spins : 0u;  // new window, new budget (a give-up sticks)
                  const uint32_t wend = ((cwi + 1) << 10) + tb;
                  for (; t + 32 <= len && t < wend; t += 32) {
                    if (dbg) ++dg[7];
                    const uint32_t r = (t - tb) & 1023u, ln = r >> 4;
                    const uint64_t sw0 = (uint64_t)readlane_u(cw.x, ln) | ((uint64_t)readlane_u(cw.y, ln) << 32);
                    const uint64_t sw1 = (uint64_t)readlane_u(cw.z, ln) | ((uint64_t)readlane_u(cw.w, ln) << 32);
                    const uint64_t sw2 = (uint64_t)readlane_u(cw.x, ln + 1) | ((uint64_t)readlane_u(cw.y, ln + 1) << 32);
                    const uint64_t sw3 = (uint64_t)readlane_u(cw.z, ln + 1) | ((uint64_t)readlane_u(cw.w, ln + 1) << 32);
                    if constexpr (DST == 2) {  // granule ring flow control, once per 32 observations
                        if (!cons_ok(uni64(cons_v), (int)t + 32 - (int)kGR + 8)) wait_cons((int)t + 32 - (int)kGR + 8);
                        if constexpr (kXh) cons_v = __hip_atomic_load(consf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        else cons_v = g_ld64(cons_out);
                    }
                    if constexpr (DST == 1 && kXh) {  // forward last iteration's load, issue the next
                        if (hrd) {
                            if (lane == 0) __hip_atomic_store(consf, cons_h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            cons_h = g_ld64(cons_out);
                        }
                    }
                    auto group = [&](auto jc, uint64_t sw) {
                        constexpr uint32_t j = decltype(jc)::value;
                        const uint32_t tg = t + 8 * j;
                        float bv = kInf;  // lanes 0..7: the previous block's last scores of tg..tg+7
                        float gl[8];      // SVH_PIPE_RING8: this group's last-slot scores
                        if constexpr (SRC == 2) {
                            if constexpr (kPfAsm) wait_vmcnt<GPF - 1>();  // gq[j]: GPF - 1 later loads in flight
                            uint64_t gv = gq[j % GPF];
                            while (!kNoWait && __builtin_amdgcn_ballot_w64((uint32_t)(gv >> 32) != gtag(ep, tg)) != 0) {
                                if (dbg) ++dg[5];
                                if (give_up()) break;
                                __builtin_amdgcn_s_sleep(1);
                                gv = g_ld64_slow(gin + ((tg + (lane & 7u)) & (kGR - 1)));
                            }
                            bv = __builtin_bit_cast(float, (uint32_t)gv);
                            prefetch(gq[j % GPF], gin + ((tg + 8 * GPF + (lane & 7u)) & (kGR - 1)));
                        }
                        if constexpr (DST == 1) {
                            if constexpr (SVH_PIPE_LDSX) asm volatile("" : "+v"(nc_rd));
                            if ((int)uniform((int)nc_rd) < (int)tg + 8 - (int)kR) wait_next((int)tg + 8 - (int)kR);
                        }
                        auto one = [&](auto kc) {
                            constexpr uint32_t k = decltype(kc)::value;
                            const uint32_t o = (uint32_t)((sw >> (8 * k)) & 0xFFu);
                            if constexpr (SRC == 1 && k == 1) {  // step 0 used only the previous vector
                                if (!next_ok) {  // the producer had not published this group: wait, re-load
                                    if (dbg) ++dg[14];
                                    uint32_t z = 0;  // SVH_PIPE_LDSX: an address the compiler cannot hoist
                                    if constexpr (SVH_PIPE_LDSX) asm volatile("v_mov_b32 %0, 0" : "=v"(z));
                                    wait_prev(tg + 8);
                                    asm volatile("" ::: "memory");
                                    bv_next = lds_ldf_slow(ring_prev + ring_idx(8 * j + (lane & 7u), 63) + z);
                                }
                            }
                            if constexpr (SRC == 1) bv = bv_next;
                            if constexpr (L2) {
                                // groups start at odd t (tb = 1): k even is a chunk's first observation,
                                // k odd its second, where the chunk runs with the previous block's
                                // scores of t - 2 (lane k - 2 of bv; k = 1: lane 7 of the previous
                                // group's) and t - 1 (lane k - 1)
                                if constexpr (k & 1u) {
                                    const uint32_t o1 = (uint32_t)((sw >> (8 * (k - 1))) & 0xFFu);
                                    if constexpr (k == 1) step2(o1, o, shr_in<7>(v[0], bv_prev), shr_in<0>(v[1], bv));
                                    else step2(o1, o, shr_in<(int)k - 2>(v[0], bv), shr_in<(int)k - 1>(v[1], bv));
                                }
                            } else if constexpr (k == 0) {
                                step(o, ChainIn<7>{bv_prev});
                            } else {
                                step(o, ChainIn<(int)k - 1>{bv});
                            }
                            if constexpr (SVH_PIPE_RING8) {  // kept for the group's two 16-byte stores
                                gl[k] = L2 ? ((k & 1u) ? v[0] : v[1]) : v[SM - 1];
                                if constexpr (k == 3 || k == 7)
                                    *reinterpret_cast<float4*>(ring_w + ring_idx(8 * j + k - 3, lane)) =
                                        make_float4(gl[k - 3], gl[k - 2], gl[k - 1], gl[k]);
                            } else {
                                ring_w[ring_idx(8 * j + k, lane)] = v[SM - 1];
                            }
                            paths_after(tg + k, std::bool_constant<j == 0 && k == 0>{},
                                        std::bool_constant<k == 0 && (j == 0 || j == 2)>{},
                                        std::bool_constant<j == 3 && k == 7>{}, std::integral_constant<uint32_t, k & 3u>{});
                            if constexpr (k == SVH_PIPE_CNTSTEP) {  // the counts checked at the end of the group
                                asm volatile("" ::: "memory");
                                if constexpr (SRC == 1) pc_rd = lds_ld32(cnt_w - 1);
                                if constexpr (DST == 1) nc_rd = lds_ld32(cnt_w + 1);
                                if constexpr (SRC == 1 && SVH_PIPE_EARLYV) {  // after the count it is checked against
                                    asm volatile("" ::: "memory");
                                    bv_spec = ring_prev[ring_idx(((8 * j + 8) & (kR - 1)) + (lane & 7u), 63)];
                                }
                                // SVH_PIPE_LDSX: issued here, not where the scheduler would sink them (the
                                // group's end, right before their use)
                                if constexpr (SVH_PIPE_LDSX) __builtin_amdgcn_sched_barrier(0);
                            }
                            if constexpr (SVH_PIPE_LDSX && SVH_PIPE_RING8 && k == 3) __builtin_amdgcn_sched_barrier(0);
                            if constexpr (DST == 2 && kGst != 0 && k == kGst) {  // the last group's granules
                                if (gpend_t && lane < 8)
                                    st_gran(gout + ((gpend_t + lane) & (kGR - 1)),
                                           ((uint64_t)gtag(ep, gpend_t) << 32) | __builtin_bit_cast(uint32_t, gpend));
                                gpend_t = 0;
                            }
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
                        asm volatile("" ::: "memory");
                        put_cnt(tg + 8);
                        if constexpr (SRC == 1) {  // the next group's boundary vector (valid if next_ok)
                            if constexpr (SVH_PIPE_LDSX) asm volatile("" : "+v"(pc_rd));
                            next_ok = kNoWait || (uint32_t)uniform((int)pc_rd) >= tg + 16;
                            asm volatile("" ::: "memory");
                            if constexpr (SVH_PIPE_EARLYV) bv_next = bv_spec;
                            else bv_next = ring_prev[ring_idx(((8 * j + 8) & (kR - 1)) + (lane & 7u), 63)];
                        }
                        if constexpr (DST == 2) {
                            // granules of the previous group (read back from the ring one group ago)
                            if constexpr (kGst == 0) {
                                if (gpend_t && lane < 8)
                                    st_gran(gout + ((gpend_t + lane) & (kGR - 1)),
                                           ((uint64_t)gtag(ep, gpend_t) << 32) | __builtin_bit_cast(uint32_t, gpend));
                            }
                            gpend = ring_w[ring_idx(8 * j + (lane & 7u), 63)];
                            gpend_t = tg;
                        }
                        if constexpr ((SRC == 2 || (SRC == 1 && kXh)) && j == 3) {
                            if ((SRC == 2 ? !helped : hpub) && lane == 0) st_cons(((uint64_t)ep << 32) | (tg + 8));
                        }
                    };
                    group(std::integral_constant<uint32_t, 0>{}, sw0);
                    group(std::integral_constant<uint32_t, 1>{}, sw1);
                    group(std::integral_constant<uint32_t, 2>{}, sw2);
                    group(std::integral_constant<uint32_t, 3>{}, sw3);
                  }
                }
                // the tail's windows; the tail's granule polls start afresh (nothing of the head's
                // stays live through the body)
                gbase = 0x80000000u;
                cwi = (t - tb) >> 10;
                cw = load_window(cwi);
                nw = load_window(cwi + 1);
                bprev = readlane_f(bv_prev, 7);
                bprev2 = readlane_f(bv_prev, 6);
                if constexpr (SRC == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the prefetches
                if constexpr (DST == 2) {
                    if (gpend_t && lane < 8)
                        st_gran(gout + ((gpend_t + lane) & (kGR - 1)),
                               ((uint64_t)gtag(ep, gpend_t) << 32) | __builtin_bit_cast(uint32_t, gpend));
                }
            }
            if (dbg) {
                const unsigned long long c1 = __builtin_amdgcn_s_memtime();
                dg[0] = c1 - c0;
                c0 = c1;
            }
            SVH_RT(10);
            // tail
            for (; t < len; ++t) single(t);
            if (dbg) dg[2] = __builtin_amdgcn_s_memtime() - c0;
            SVH_RT(11);
            if constexpr (PATHS) {
                // rows the loop did not store: masks of rows below len-1 past the last full word,
                // ring rows of the last partial group of 32
                const uint32_t mdone = (len - 1) & ~31u;
                if (mdone < len - 1) store_masks(mdone >> 5, len - 1 - mdone);
                if (((len - 1) & 31u) != 31u) reduce_ring((len - 1) & ~31u, len);
            }
        };

        if (FLOOR) {
            if (len > first) sweep(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
        } else if (len > first && dbg && (m.diag & 1u)) {
            sweep(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});  // no exchange (timing only)
        } else if (len > first) {
            using I0 = std::integral_constant<int, 0>;
            using I1 = std::integral_constant<int, 1>;
            using I2 = std::integral_constant<int, 2>;
            switch (src * 3 + dst) {
                case 0: sweep(I0{}, I0{}); break;
                case 1: sweep(I0{}, I1{}); break;
                case 2: sweep(I0{}, I2{}); break;
                case 3: sweep(I1{}, I0{}); break;
                case 4: sweep(I1{}, I1{}); break;
                case 5: sweep(I1{}, I2{}); break;
                case 6: sweep(I2{}, I0{}); break;
                case 7: sweep(I2{}, I1{}); break;
                default: sweep(I2{}, I2{}); break;
            }
        }
        if (dbg && lane == 0)
            for (int k = 0; k < kPipeStamps; ++k) m.stamps[((size_t)id * W + w) * kPipeStamps + k] = dg[k];
        if (spins > kSpinLimit && lane == 0 && b.fault) atomicOr(b.fault, kFaultPipe);

        // ---- scores of the light positions and this wave's partials
        float* out = b.scores + (size_t)q * m.n;
        float bvv = kInf;
        uint32_t bk = kNoRow;
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            const uint32_t r = m.lrow[p0 + s];
            if (r != kNoRow) {
                if (PATHS || L2) out[r] = v[s];
                else g_st_score(out + r, v[s]);  // the row's re-run may come from another XCD
                lex_min(bvv, bk, v[s], r);
            }
        }
        wave_lexmin63(bvv, bk);
        const float cmin = wave_min63(CF.x);
        const bool any_viol = __builtin_amdgcn_ballot_w64(viol != 0) != 0;  // all lanes active here
        if (lane == 63) {
            red[w * 4 + 0] = cmin;
            red[w * 4 + 1] = bvv;
            red[w * 4 + 2] = __builtin_bit_cast(float, bk);
            red[w * 4 + 3] = __builtin_bit_cast(float, any_viol ? 1u : 0u);
        }
    } else if (lane == 63) {
        red[w * 4 + 0] = kInf;
        red[w * 4 + 1] = kInf;
        red[w * 4 + 2] = __builtin_bit_cast(float, kNoRow);
        red[w * 4 + 3] = 0.0f;
    }
    __syncthreads();

    // ---- per-sequence combine (the workgroup that finishes the sequence last) and launch end
    if (tid == 0) {
        float cm = kInf, bvv = kInf;
        uint32_t bk = kNoRow, vi = 0;
        bool rr = false;
        for (uint32_t u = 0; u < (uint32_t)W; ++u) {
            cm = fminf(cm, red[u * 4 + 0]);
            lex_min(bvv, bk, red[u * 4 + 1], __builtin_bit_cast(uint32_t, red[u * 4 + 2]));
            vi |= __builtin_bit_cast(uint32_t, red[u * 4 + 3]);
        }
        uint64_t* part = x.part + ((size_t)q * G + g) * 2;
        g_st64(part, ((uint64_t)vi << 32) | __builtin_bit_cast(uint32_t, cm));
        g_st64(part + 1, lex_key(bvv, bk));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t d = __hip_atomic_fetch_add(x.done + q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == G - 1) {
            float C = kInf;
            uint64_t key = ~0ull;
            vi = 0;
            for (uint32_t u = 0; u < G; ++u) {
                const uint64_t* pu = x.part + ((size_t)q * G + u) * 2;
                const uint64_t a = g_ld64(pu), k2 = g_ld64(pu + 1);
                C = fminf(C, __builtin_bit_cast(float, (uint32_t)a));
                vi |= (uint32_t)(a >> 32);
                key = k2 < key ? k2 : key;
            }
            float* out = b.scores + (size_t)q * m.n;
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
            rr = !PATHS && !L2 && !FLOOR && m.rerun && vi;  // this workgroup re-runs the row (below)
        }
        *tick = rr ? 1u : 0u;  // (the ticket itself is in id since the first barrier)
    }
    if constexpr (!PATHS && !L2) {
        if (m.rerun) {
            __syncthreads();
            if (*tick == 1u) pipe_rerun_row<SM, W, SX>(m, b, q, lds);
        }
    }
    if (tid == 0) {
        const uint32_t f = __hip_atomic_fetch_add(x.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (f == gridDim.x - 1) pipe_reset_counters(x);  // every workgroup has taken its ticket
    }
}

}  // namespace

// The kernel's instantiations live in three translation units (they compile in parallel):
// pipe.hip TM = 0 (every geometry, decoded-path variants at 2 x 4), pipe_tm1.hip TM = 1..4 (2 slots,
// 4 waves), pipe_tm1p.hip TM = 1 / 4 decoded-path variants (2 x 4).  Each returns the kernel for
// (slots, waves, sx, PATHS, ties_heavy) or nullptr.
const void* pipe_kernel_tm0(int sm, int waves, bool sx, int paths);
const void* pipe_kernel_tm1(int sm, int waves, bool sx, int paths);
const void* pipe_kernel_tm1_paths(int sm, int waves, bool sx, int paths, int tm);
const void* pipe_kernel_floor(bool sx);

}  // namespace svh
