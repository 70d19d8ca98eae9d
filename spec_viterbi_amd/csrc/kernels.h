// Internal interface between the host runtime (model.cpp) and the HIP kernels.
// Not part of the public ABI (that is include/svh.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace svh {

constexpr int kMaxHeavy = 4;      // heavy rows a fused-kernel family can hold
constexpr int kMaxExc = 4;        // exception terms per heavy row
constexpr int kMaxWaves = 16;     // waves per workgroup (B <= 1024)
constexpr uint32_t kNoPred = 0xFFFFu;
constexpr uint32_t kSymChunk = 4096;  // symbols staged in LDS per refill
constexpr uint32_t kSymPad = 64;      // zero bytes after every sequence in device memory
constexpr int kMaxFusedThreads = 512;

enum HeavyMode : int { kHeavyGeneral = 0, kHeavyUniform = 1 };

// Register-resident schedule of the fused step kernel (built by Plan in model.cpp).
//   State j of the model lives in slot s = j / B of thread t = j % B (strided, so a wave's LDS
//   accesses to v are lane-consecutive and bank-conflict free).  LDS index space of one score
//   buffer: [0, estride) states, estride = +inf scratch, estride+1+h = heavy row h.
struct FusedModel {
    const float* emis;      // [S][estride] fp32, +inf padding beyond n (+16 floats)
    const float* start;     // [estride] dense start column, +inf where absent
    const uint32_t* lcol;   // [(s*R + r)*B + t] light-row term source (LDS index)
    const float* lval;      // [(s*R + r)*B + t] light-row term T^T value (+inf padding)
    const float* hval;      // GENERAL: [(h*SM + s)*B + t] heavy-row T^T over own sources
    const uint8_t* hvalid;  // GENERAL: same layout, 1 where T^T has the entry (paths)
    const float* hmask;     // UNIFORM: [s*B + t] 0 if own source is in the shared set U, +inf
    int hrow[kMaxHeavy];    // heavy row ids (dummies: estride)
    float hw[kMaxHeavy];    // UNIFORM: dominant weight of heavy row h
    uint32_t xk[kMaxHeavy][kMaxExc];  // exception term source (LDS index; scratch = none)
    float xw[kMaxHeavy][kMaxExc];     // exception term weight (+inf = none)
    uint32_t H;             // number of real heavy rows
    uint32_t n;             // states
    uint32_t S;             // symbols
    uint32_t slots;         // SM: slots per thread (the kernel instantiation)
    uint32_t estride;       // slots * B (>= n)
    uint32_t vstride;       // floats per LDS score buffer (multiple of 4)
    uint32_t B;             // threads per workgroup
};

// Bits of FusedBatch::fault.
constexpr uint32_t kFaultPipe = 1u, kFaultPipeWide = 2u, kFaultChain = 4u;

// One batch of sequences.  Symbols are uint8; each sequence 16-byte aligned, kSymPad padded.
struct FusedBatch {
    const uint8_t* symbols;
    const uint64_t* sym_off;   // [nseq] byte offset of sequence q
    const uint32_t* begin;     // [nseq] first step to run (0: start from the start column)
    const uint32_t* end;       // [nseq] sequence length (steps run: max(begin,1)..end-1)
    const float* v_in;         // rows of initial scores when begin > 0
    const uint32_t* v_in_row;  // [nseq] row of v_in for sequence q (stride n)
    float* scores;             // [nseq][n] final scores
    int64_t* best;             // [nseq] lowest-index argmin of final scores (nullable)
    uint16_t* bp;              // backpointers (PATHS only)
    const uint64_t* bp_off;    // [nseq] element offset of sequence q's (len-1) x n block
    // Chain-kernel decoded paths (chain.hip): per backpointer row r (observation r+1)
    //   cmask: bit = "light position took its heavy term"; u32 words [r/32][slot][thread], bit
    //          31 - r%32 of a word is row r (position thread*SM + slot)
    //   hrec:  [r][kRecWords] u32: [0..1] the heavy scores of observation r (f32), [2] the light
    //          minimum of observation r (f32); the traceback re-evaluates the heavy rows' argmin
    //          from these (chain_paths.hip)
    //   ckpt:  the light scores of every kCkptEvery-th observation ([c / kCkptEvery][SM * B],
    //          slot-major like the model tables): the traceback recomputes a row's light scores
    //          from the checkpoint below it where it needs the light-set argmin j*
    uint32_t* cmask;
    const uint64_t* cmask_off;  // [nseq] u32 offset of sequence q's masks
    uint32_t* hrec;
    const uint64_t* hrec_off;   // [nseq] u32 offset of sequence q's records
    float* ckpt;
    const uint64_t* ckpt_off;   // [nseq] float offset of sequence q's checkpoint rows
    // Pipelined-kernel decoded paths (pipe.hip PATHS, pipe_paths.hip): cmask / ckpt / hrec above
    // in the pipelined plan's layouts (kernels.h, PipeModel), plus
    //   prec: [blk][half][t] per-block partial records {min of the half-wave's light scores at
    //         t-1, min of its sink partials at t} for observations t in [1, len); the traceback
    //         kernel folds them into hrec rows {F, C, mu}
    //   fck:  F's score at every 32nd observation (F(32k)), written by block 0
    float2* prec;
    const uint64_t* prec_off;   // [nseq] float2 offset of sequence q's partial records
    float* fck;
    const uint64_t* fck_off;    // [nseq] float offset of sequence q's F checkpoints
    // Fallback pass after the pipelined kernel (pipe.hip): when set, only rows with
    // run_mask[q] != 0 run (the others return at once).  Step kernels check it first.
    const uint32_t* run_mask;
    const struct PipeScratch* pipe;  // host side only: scratch of the pipelined kernel (nullable)
    // The batch's own fault word (nullable): a kernel whose bounded wait gave up ORs its bit in
    // (kFaultPipe, kFaultPipeWide, kFaultChain); the batch that ran it reports and clears it.
    uint32_t* fault;
    uint32_t nseq;
};

// Chain ("band") kernel model: the MSV shape of every reference .chmm (N, M_1..M_L, C).
//   Light rows (all but <= kBandHeavy heavy rows), in ascending row order at positions p, have
//   terms only from heavy rows (weights aw) and from the light row at position p-1 (weight bw).
//   Each heavy row h has one weight w_h shared by ALL light rows (or no light source at all) plus
//   terms from heavy rows.  Position p = t*SM + s lives in slot s of thread t (blocked); per-thread
//   tables use the lane-consecutive index s*B + t.
constexpr int kBandHeavy = 2;
constexpr int kMaxBandThreads = 1024;
constexpr int kDefaultBandThreads = 512;
// Row tail (floats at offset SM*B of every emission row of symbol o):
//   cA[h]    = fl(E_o[h] + w_h)          the shared uniform term of heavy row h
//   cX[h][k] = fl(E_o[h] + T^T[h][k])    heavy row k -> heavy row h (+inf if absent)
//   Eh[h]    = E_o[h]
constexpr int kBandTailA = 0;
constexpr int kBandTailX = kBandHeavy;
constexpr int kBandTailE = kBandHeavy + kBandHeavy * kBandHeavy;
constexpr int kBandTail = 8;  // floats (>= kBandTailE + kBandHeavy, multiple of 4)
// X[h][k] (heavy row k -> heavy row h) in the tail: diagonal pair first, then the off-diagonal
// pair, so each is one aligned f32 pair for v_pk_add_f32: [A0 A1 | X00 X11 | X01 X10 | E0 E1].
constexpr int band_tail_x(int h, int k) { return kBandTailX + (h == k ? h : kBandHeavy + h); }
static_assert(kBandHeavy == 2, "band_tail_x assumes two heavy rows");
static_assert(kBandTailE + kBandHeavy <= kBandTail, "band row tail");

struct BandModel {
    const float* erows;     // [S][erow]: [s*B + t] = E[o][row of position t*SM+s] (+inf pad), tail
    const float* erows_t;   // chain kernel, streamed E: [S][B][round_up(SM,4)] (+inf pad)
    const float* start;     // [SM*B] start of light positions (+inf pad)
    const float* aw;        // [HA][SM*B] weight of the term from heavy row h
    const float* bw;        // [SM*B] weight of the term from position p-1
    const uint32_t* lrow;   // [SM*B] row id of the position (0xFFFFFFFF pad)
    int hrow[kBandHeavy];   // heavy row ids (dummy rows: hvalid 0)
    int hvalid[kBandHeavy];
    float hstart[kBandHeavy];
    uint32_t n, S, B, SM, erow, H;
    uint32_t ge;  // chain kernel: 1 = emission rows streamed from L2 (erows_t), 0 = held in VGPRs
    uint32_t dbg;  // diagnostic ablations (timing only, wrong results): 1 no DMA, 2 no barrier,
                   // 4 s_memtime segment stamps into `stamps`, 8 no s_sleep in spins,
                   // 16 chain kernel ignores the exchange tags (never waits)
    unsigned long long* stamps;  // [nseq][kMaxWaves][kBandStamps] cycle sums (dbg & 4)
    // decoded paths (chain kernel, HA <= 1):
    const uint8_t* pflags;  // [SM*B] bit0: term from position p-1 exists, bit1: term from heavy
                            // row 0 exists, bit2: heavy row 0 < row of p-1 (heavy wins ties)
    const int32_t* spos;    // [n] position of a light row, -1-h for heavy row h
    uint32_t hx_exist;      // bit h*kBandHeavy+k: heavy row k -> heavy row h term exists
    uint32_t hl_exist;      // bit h: heavy row h has the shared term from every light row
    uint32_t ties_heavy;    // 1: every light position with a heavy term has it win ties (one
                            // compare per mask bit)
};
constexpr int kBandStamps = 8;

// Barrier-free chain kernel (chain.hip): emission table in VGPRs (S <= kChainMaxSym), waves
// synchronise through tagged 64-bit LDS words instead of s_barrier.
constexpr int kChainMaxSym = 32;
constexpr int kChainMaxThreads = 512;
constexpr uint32_t kChainSymChunk = 32768;  // symbols staged in LDS per refill
constexpr int kChainRing = 8;  // exchange ring depth (observations in flight between waves)
inline size_t chain_lds_bytes() {
    // heavy constants | tagged records [ring][waves][2] u64 | cells, counts, junk [ring] 4 B each |
    // reduction | staged symbols
    return (size_t)kChainMaxSym * kBandTail * sizeof(float) + (size_t)kChainRing * 2 * kMaxWaves * 8 +
           3 * kChainRing * 4 + 2 * kMaxWaves * sizeof(float) + kChainSymChunk;
}
// Chain kernel for (SM slots, W waves, HA heavy feeders, E streamed?); false if not instantiated.
bool chain_supported(int sm, int waves, int ha, bool ge);
// Decoded-path variant (E in VGPRs, HA <= 1) instantiated for this geometry?
bool chain_paths_supported(int sm, int waves);
// b.cmask != nullptr selects the decoded-path variant (every sequence must start at step 0).
hipError_t launch_chain(const BandModel& m, int ha, const FusedBatch& b, hipStream_t stream);
// Path traceback over the chain kernel's compact backpointers (one wave per sequence).
hipError_t launch_chain_traceback(const BandModel& m, const FusedBatch& b, const uint64_t* path_off,
                                  int32_t* paths, hipStream_t stream);
// u32 mask words / u32 records the decoded-path variant writes for a sequence of length len.
inline uint64_t chain_mask_words(uint64_t len, uint32_t waves, uint32_t sm) {
    return len > 1 ? (len - 1 + 31) / 32 * (uint64_t)sm * 64 * waves : 0;
}
// Decoded-path staging in LDS beyond chain_lds_bytes(): the heavy-record ring (rows).
constexpr uint32_t kPathRing = 64;
constexpr uint32_t kRecWords = 4;
inline size_t chain_path_lds_bytes() { return (size_t)kPathRing * kRecWords * 4; }
inline uint64_t chain_hrec_words(uint64_t len) { return len > 1 ? (len - 1) * kRecWords : 0; }
// Light-score checkpoints of the decoded-path variant: rows 0, kCkptEvery, ... <= len-1.
constexpr uint32_t kCkptEvery = 16;
inline uint64_t chain_ckpt_floats(uint64_t len, uint32_t sm, uint32_t threads) {
    return len ? ((len - 1) / kCkptEvery + 1) * (uint64_t)sm * threads : 0;
}

// Pipelined chain kernel (pipe.hip): MSV-shaped models whose one heavy feeder F (the rows' N) and
// sink S (C) satisfy: light rows take terms from position p-1 and from F only; F from the light
// rows (one shared weight) and itself; S from the light rows (one shared weight), itself and F.
// F's light term is speculated away -- F'(t) = fl(X_FF(o_t) + F'(t-1)) -- which removes the
// per-observation all-position reduction from the recurrence: a sequence's positions are cut
// into blocks of 64*SM that run as a pipeline of waves (each wave sweeps every observation of
// its block and streams its last position's score to the next block's wave: LDS within a
// workgroup, 8-byte tagged granules through L2 between workgroups).  Every lane checks the
// speculation exactly at every observation (fl(A_F(o_t) + min of its light scores at t-1) <
// F'(t) would have changed F); a sequence that fails it is re-run by the serial chain kernel.
// S is exact without any reduction: its update is monotone in the light scores, so
// S(t) = min over lanes of a per-lane S recurrence driven by the lane's own scores.
constexpr int kPipeRing = 32;       // LDS ring (observations) between the waves of a workgroup
constexpr int kPipeGroup = 8;       // observations per exchange group
constexpr int kPipeGRing = 256;     // L2 granule ring (observations) between workgroups
constexpr int kPipeAhead = 4;       // granule groups a consumer keeps in flight
constexpr int kPipeWindow = 1024;   // symbols per VGPR window (64 lanes x 16 B)
struct PipeModel {
    const float2* tab;      // [nblk][S][SM][64]: (fl(E_o[p] + bw_p), fl(E_o[p] + aw_p)), +inf pad
    const float* e0;        // [S][P]: E_o[row of position p] (the first observation)
    const float* start;     // [P]: start score of position p (+inf pad)
    const uint32_t* lrow;   // [P]: row id of position p (0xFFFFFFFF pad)
    const float* hc;        // [S][8]: A_S A_F X_SS X_FF | X_SF E_F E_S 0 (fl(E_o[h] + w) each)
    int rowF, rowS;         // heavy rows (rowS < 0: the model has no sink row)
    float startF, startS;
    uint32_t n, S, P, nblk, SM, W, G;  // P = nblk*64*SM positions, G workgroups per sequence
    uint32_t cus;           // wide plan: CUs of the device (W = waves per workgroup at most)
    uint32_t sx;            // S has a term from F
    uint32_t tm;            // latency plan's table mode (pipe_kernel.h): 1 = pair tables (SM = 2, S <= 20)
    uint32_t wide;          // 1: the wide plan's geometry and table layout (pipe_wide_kernel.h)
    float emax2;            // _spec level 2 on this plan (pipe_l2.hip): the largest finite ea over
                            // positions and symbols (its margin check), +inf: level 2 not supported
    // diagonal plan (diag.hip): the table [S][64 nrng] float2 {ea_p(o), eb_p(o)} of positions 0 .. 64 nrng - 1
    // in chain order (+inf past the light rows), nrng ranges of 64 diagonals per sequence; null: no plan
    const float2* dtab;
    uint32_t nrng;
    uint32_t rerun;         // latency plan, scores: a row whose speculation fails is re-run exactly by
                            // its combining workgroup (pipe_rerun_row; needs 2P + 2W floats of the ring's
                            // LDS), so no fallback launch follows the pass; 0: the host launches one
    // decoded paths (pipe PATHS variant + pipe_traceback_kernel):
    const uint8_t* pflags;  // [P] bit0: term from position p-1 exists, bit1: term from F exists,
                            // bit2: F's row < row of p-1 (F wins ties)
    const int32_t* spos;    // [n] position of a light row, -1 for F, -2 for S
    uint32_t hx_exist;      // BandModel::hx_exist (heavy x: 0 = F, 1 = S)
    uint32_t hl_exist;      // BandModel::hl_exist
    uint32_t ties_heavy;    // every light position with an F term has it win ties
    unsigned long long* stamps;  // diagnostics (SVH_PIPE_DEBUG): [ticket][W][8] counters, or null
    uint32_t diag;               // diagnostics with stamps (SVH_PIPE_DEBUG bits > 1): 1 = no boundary
                                 // exchange (every wave runs as block 0; timing only, wrong results)
};
constexpr int kPipeStamps = 15;  // written only by -DSVH_PIPE_DIAG builds of pipe.hip
// Per-batch scratch of the pipelined kernel (sized for `rows` rows).
constexpr uint32_t kCtrClass = 4, kCtrLeft = 12, kCtrWords = 16;
struct PipeScratch {
    uint32_t* ctr;    // [kCtrWords]: [0] workgroup ticket, [1] finished workgroups, [2] last epoch,
                      // [kCtrClass + r] per-class tickets (r < 8), [kCtrLeft] leftover tickets (x.xmap)
    uint32_t* done;   // [rows] finished workgroups of row q (reset by its last one)
    uint64_t* part;   // [rows][G][2]: {C min | violation, (best value, best row) key}
    uint64_t* gran;   // [rows][G-1][kPipeGRing] tagged boundary granules {score, tag}
    uint32_t* cons;   // [rows][G] granules received by workgroup g's first wave
    uint32_t* viol;   // [rows] 1: speculation failed, row needs the serial kernel
    uint32_t* xcc;    // [rows][G] (epoch << 4) | XCC id of workgroup g of row q (XCD-local hand-offs)
    uint32_t xmap;    // launch: 1 = (row, workgroup) from per-XCD-class tickets (pipe_kernel.h)
    uint32_t rows, G;
};
constexpr uint32_t kPairSymbols = 20;  // pipe_kernel.h kPairSym: the pair tables' symbol capacity
__host__ __device__ inline size_t pipe_lds_bytes(uint32_t W, uint32_t S) {
    // boundary ring [W][kPipeRing][64] | counters [16] | heavy constants [S][8] | reduction [W][4] | ticket
    return ((size_t)W * kPipeRing * 64 + 16 + (size_t)S * 8 + (size_t)W * 4 + 4) * 4;
}
// The latency plan's in-kernel re-run (PipeModel::rerun) keeps v[2][P] and red[2][W] in the ring.
__host__ __device__ inline bool pipe_rerun_fits(uint32_t P, uint32_t W) {
    return 2ull * P + 2ull * W <= (size_t)W * kPipeRing * 64;
}
bool pipe_supported(int sm, int waves, bool sx);
// table mode tm (pipe_kernel.h TM) compiled into this build at the default geometry (TM 1..3 and
// the other geometries only in SVH_PIPE_AB_ALL builds)
bool pipe_tm_supported(int tm);
// b.cmask != nullptr selects the decoded-path variant (every sequence must start at step 0).
// step_floor: the FLOOR variant (pipe_kernel.h; TM 4 geometry only): the sweep without any exchange,
// for svh_batch_step_floor_ms (b's outputs must be scratch)
hipError_t launch_pipe(const PipeModel& m, const FusedBatch& b, const PipeScratch& x, hipStream_t stream,
                       bool step_floor = false);
// _spec level 2 on the latency plan's geometry (pipe_l2.hip: pipe_kernel.h with L2): every chunk of
// two observations of every row, from observation 0, into b.scores (dense rows; best states when
// b.best); rows whose speculation fails are flagged in x.viol (re-run by spec2_kernel, runtime.cpp).
hipError_t launch_pipe_l2(const PipeModel& m, const FusedBatch& b, const PipeScratch& x, hipStream_t stream);
bool pipe_l2_supported(const PipeModel& m);
bool pipe_paths_supported(int sm, int waves);
// Decoded paths of the pipelined plan: the records {F, C, mu} from the per-block partials, then
// the path walk (pipe_paths.hip); rows with skip[q] != 0 (re-run by the chain kernel) are left
// to the chain traceback.
hipError_t launch_pipe_traceback(const PipeModel& m, const FusedBatch& b, const uint64_t* path_off, int32_t* paths,
                                 const uint32_t* skip, hipStream_t stream);
// Light positions the pipelined traceback stages in LDS (pipe_paths.hip): plans with more decode
// paths on the chain kernel.
constexpr uint32_t kPipeTbMaxP = 2560;
// Per-sequence sizes of the decoded-path buffers of the pipelined plan.
inline uint64_t pipe_mask_words(uint64_t len, uint32_t nblk, uint32_t sm) {
    return len > 1 ? (len - 1 + 31) / 32 * (uint64_t)nblk * sm * 64 : 0;
}
// heavy partials per block and observation: 2 (latency plan: one per half-wave), 1 (wide plan)
// heavy partials per block and observation: 1 on both plans (the latency plan folded its ring per
// half-wave into 2 until round 4)
__host__ __device__ inline uint32_t pipe_prec_parts(bool wide) { (void)wide; return 1u; }
inline uint64_t pipe_prec_count(uint64_t len, uint32_t nblk, uint32_t parts) { return (uint64_t)nblk * parts * len; }
inline uint64_t pipe_ckpt_floats(uint64_t len, uint32_t P) { return len ? ((len - 1) / kCkptEvery + 1) * (uint64_t)P : 0; }
inline uint64_t pipe_fck_floats(uint64_t len) { return len ? (len - 1) / 32 + 1 : 0; }
// LDS of the decoded-path variant beyond pipe_lds_bytes: a ring of 32 rows {pm, c} per wave
constexpr uint32_t kPRingStride = 132;  // floats per row: 64 lanes x 2 + 4 padding (bank spread)
// Latency plan (pipe_kernel.h PATHS): per wave 8 quads (4 observations each); a quad is two planes
// (observations 0-1, 2-3) of 64 lanes x float4, planes kPPlane and quads kPQuadStride floats apart:
// each 16-byte store of a plane is contiguous over the lanes (conflict-free), and the transposed
// fold's 32 (quad, observation) addresses for one source lane are 8q + 4 (r / 2) + 2 (r % 2) mod 64
// dwords, every bank pair once.  (Round 5: the ring's stores cost 50 us of the 0.37 ms path kernel,
// -DSVH_PIPE_NOPRING; the layout before, lanes' 32 bytes side by side in 584 floats per quad, put
// each 16-byte store on half the banks.  This layout measured the same -- forward kernels
// 0.367-0.375 ms against 0.364-0.372, profiles/r05_paths/ab_planar.log -- so the stores' cost is
// not bank conflicts; kept for its smaller footprint, 16.6 against 18.7 KB per wave.)
constexpr uint32_t kPPlane = 260;       // floats: 64 x 4 + 4 (260 = 4 mod 64)
constexpr uint32_t kPQuadStride = 520;  // floats: two planes (520 = 8 mod 64)
inline size_t pipe_path_lds_bytes(uint32_t W) { return (size_t)W * 8 * kPQuadStride * 4; }
// Diagonal plan (diag.hip): the latency plan's recurrence with every lane on an anti-diagonal of the
// (position, observation) grid -- lane l of range r holds position (64 r + l + i) mod (64 nrng) after
// step i, so a position's chain input is the lane's own previous score (no exchange between waves).
// A workgroup is diag_waves_for(nseq) sequences x one range; rows whose speculation fails are re-run
// in the same launch.  Scores only; a row starts at observation 0 or resumes at begin > 0 from v_in.
uint32_t diag_waves_for(uint64_t nseq);
size_t diag_lds_bytes(uint32_t W, uint32_t S, uint32_t P);
hipError_t launch_diag(const PipeModel& m, const FusedBatch& b, const PipeScratch& x, hipStream_t stream);

// Wide pipelined plan (pipe_wide.hip): one block of 64*SM positions per workgroup, W sequences
// (one per wave), the block's table [nblk][S][NC][64] float4 in LDS (PipeModel.tab; G = nblk);
// NC = SM/2 (eb|ea) chunks + {A_S A_F X_SS X_FF} [+ {X_SF 0 0 0} when sx], constants per lane.
__host__ __device__ inline uint32_t pipew_chunks(uint32_t SM, bool sx) { return SM / 2 + 1 + (sx ? 1 : 0); }
inline size_t pipew_lds_bytes(uint32_t SM, uint32_t W, uint32_t S, bool sx, bool paths = false) {
    // table [S][NC][64] float4 | boundary ring [W][8][64] | ticket | paths: ring [W][8][kPRingStride]
    return (size_t)S * pipew_chunks(SM, sx) * 64 * 16 + (size_t)W * 8 * 64 * 4 + 16 +
           (paths ? (size_t)W * 8 * kPRingStride * 4 : 0);
}
bool pipew_supported(int sm, int waves, bool sx);
// Decoded paths on the wide plan: the most sequences per workgroup whose LDS fits (0: none).
uint32_t pipew_paths_waves_max(uint32_t sm, uint32_t S, bool sx);
bool pipew_paths_supported(int sm, uint32_t S, bool sx);
// Sequences (waves) per workgroup of a wide launch over nseq rows: the fewest of 1, 2, 4, 8, 12,
// 16 that give about one workgroup per CU (a workgroup holds a CU's LDS), at most m.W.
inline uint32_t pipew_waves_for(const PipeModel& m, uint64_t nseq) {
    const uint64_t need = (nseq * m.nblk + m.cus - 1) / (m.cus ? m.cus : 1);
    static const uint32_t ws[] = {1, 2, 4, 8, 12, 16};
    uint32_t w = m.W;
    for (uint32_t c : ws)
        if (c >= need) {
            w = c < m.W ? c : m.W;
            break;
        }
    return w;
}
// b.cmask != nullptr selects the decoded-path variant (every sequence must start at step 0).
hipError_t launch_pipew(const PipeModel& m, const FusedBatch& b, const PipeScratch& x, hipStream_t stream);

// CSR of T^T used by the generic kernel and the _spec precompute.
struct CsrModel {
    const float* emis;       // [S][n]
    const float* start;      // [n]
    const uint32_t* rowptr;  // [n + 1]
    const uint32_t* col;     // [nnz]
    const float* val;        // [nnz]
    const uint32_t* row_of;  // [nnz] row of entry p
    uint32_t n;
    uint32_t S;
    uint32_t nnz;
};

// Kernel families of the fused step kernel.
enum FusedFamily : int {
    kFamR2Uni = 0,  // R=2, HM=2, uniform heavy rows (MSV / HMMER-style models)
    kFamR2 = 1,     // R=2, HM=2, general heavy rows
    kFamR4 = 2,     // R=4, HM=4
    kFamR8 = 3,     // R=8, HM=4
    kFamR16 = 4,    // R=16, HM=4
    kNumFamilies = 5
};
int family_rmax(int fam);
int family_hmax(int fam);
int family_xmax(int fam);
int family_mode(int fam);
constexpr int kSlotChoices[] = {1, 2, 3, 4, 5, 6, 8, 10, 12, 16};
constexpr int kNumSlotChoices = 10;

// Per-family kernel lookup (fused_r*.hip).
const void* fused_kernel_r2uni(int smax, bool paths);
const void* fused_kernel_r2(int smax, bool paths);
const void* fused_kernel_r4(int smax, bool paths);
const void* fused_kernel_r8(int smax, bool paths);
const void* fused_kernel_r16(int smax, bool paths);

// LDS bytes the fused kernel needs for (SM, B, vstride): 3 score buffers, 3 E-ring slots of
// ceil(SM/4) 16-byte DMA rows, heavy keys, reduction scratch, symbol ring.
inline size_t fused_lds_bytes_for(int sm, uint32_t B, uint32_t vstride) {
    const size_t ndma = (size_t)(sm + 3) / 4;
    return (3 * (size_t)vstride + 3 * ndma * B * 4) * sizeof(float) +
           3 * kMaxHeavy * sizeof(uint64_t) + 2 * kMaxWaves * sizeof(float) + kSymChunk + 64 + 16;
}
inline size_t fused_lds_bytes(const FusedModel& m) {
    return fused_lds_bytes_for((int)m.slots, m.B, m.vstride);
}
constexpr size_t kMaxLdsBytes = 160 * 1024;

hipError_t launch_fused(const FusedModel& m, const FusedBatch& b, int fam, bool paths,
                        hipStream_t stream);
// Chain kernel (band.hip): slot counts instantiated, LDS bytes, launcher.
constexpr int kBandSlotChoices[] = {1, 2, 3, 4, 5, 6, 8, 10, 12, 16};
constexpr int kNumBandSlotChoices = 10;
inline size_t band_lds_bytes(uint32_t erow) {
    return (3 * (size_t)erow + 4 * kMaxWaves + 2 * kMaxWaves) * sizeof(float) + kSymChunk + 64 + 16;
}
hipError_t launch_band(const BandModel& m, int ha, const FusedBatch& b, hipStream_t stream);
size_t generic_lds_bytes(uint32_t n);
hipError_t launch_generic(const CsrModel& m, const FusedBatch& b, int threads, bool paths,
                          hipStream_t stream);
hipError_t launch_traceback(const FusedBatch& b, const uint64_t* path_off, int32_t* paths,
                            uint32_t n, hipStream_t stream);

// _spec precompute / run (reference: GraphBLAS_spec_impl.cpp:15-36, 50-97, 146-181).
// Dense products are stored row-major with row stride pstride = round_up(n, 4) (+inf padding).
// K2: mfold[p * S + i] = fl(E[i][row(p)] + val[p])   (M_i = diag(E_i) (x) T^T, per nnz)
hipError_t launch_spec_fold(const CsrModel& m, float* mfold, hipStream_t stream);
// Dense level-1 products H1[o][j][m] (+inf off-pattern).
hipError_t launch_spec_densify(const CsrModel& m, const float* mfold, float* h1, uint32_t pstride,
                               hipStream_t stream);
// K3: H_new[kp * S + i][j][m] = min_p fl(M_i[j][p] + H_prev[kp][p][m]) for kp in [0, kprev).
hipError_t launch_spec_extend(const CsrModel& m, const float* mfold, const float* h_prev,
                              uint64_t kprev, float* h_new, uint32_t pstride, hipStream_t stream);
// K4: one level-L chunk for every sequence with chunk < nchunks[q].
struct SpecChunkBatch {
    const uint8_t* symbols;
    const uint64_t* sym_off;
    const uint32_t* nchunks;
    const float* v_src;  // [nseq][n]
    float* v_dst;        // [nseq][n]
    uint32_t nseq;
    uint32_t level;
    uint32_t chunk;
};
hipError_t launch_spec_chunk(const CsrModel& m, const float* products, const SpecChunkBatch& c,
                             uint32_t pstride, hipStream_t stream);
// _spec level 2 on chip (spec2.hip): one persistent workgroup of kSpec2Threads per sequence runs
// every chunk of two observations from the folded sparse matrices (no dense products).
// Rows with at most kSpec2LightMax terms are light (their terms in registers of the thread
// r % 1024, slot r / 1024); the others heavy (their terms padded to a multiple of nhs and spread
// over consecutive threads, nhs per thread, one row per thread).  Per term two words: `a` where the
// column's score is read in LDS (float index; bit 31: a heavy row's order-preserving key) and `b`
// where the column's (b, v) pair list starts (bits 0..19, pair index) and which count cell holds
// its length (bits 20..31: heavy index, H = KL for a light column, H + 1 = 0 for padding).
constexpr uint32_t kSpec2Threads = 1024;
constexpr uint32_t kSpec2LightMax = 4;
struct Spec2Model {
    const float* emis;     // [S][n]
    const uint32_t* la;    // [R][KL][1024] light terms: score address
    const uint32_t* lb;    // [R][KL][1024] light terms: pair list
    const float* lv;       // [R][KL][1024] light terms: T^T value (+inf: padding)
    const uint32_t* thr;   // [1024] heavy row of the thread (H: none)
    const uint32_t* tcp;   // [1024] pair index of that row's candidate range
    const uint32_t* ha;    // [1024][NHS] heavy terms: score address
    const uint32_t* hb;    // [1024][NHS] heavy terms: pair list
    const float* hv;       // [1024][NHS] heavy terms: T^T value (+inf: padding)
    const uint32_t* hrow;  // [H] state of heavy row h
    const float* amax;     // [H] max over symbols and out-terms (j, p) of the finite fl(E_s[j] + T^T[j][p])
    uint32_t n, S, H, NP;  // NP: candidate pair capacity (the heavy rows' padded term counts)
    uint32_t R, KL, NHS;   // instantiated sizes (rounded: 2/3/4, 2/4, 4/6/8)
    uint32_t nhs;          // heavy terms per thread (<= NHS)
    uint32_t prune;        // every score >= 0: candidates pruned (spec2.hip); 0: every term kept
    unsigned long long* stamps;  // diagnostics (-DSVH_SPEC2_DIAG builds, SVH_SPEC2_DEBUG=1): [seq][16][8]
};
constexpr int kSpec2Stamps = 8;
struct Spec2Batch {
    const uint8_t* symbols;
    const uint64_t* sym_off;
    const uint32_t* len;      // [nseq] sequence lengths
    const uint32_t* nchunks;  // [nseq] floor((len - 1) / 2)
    float* v;                 // [nseq][n] in: the state after observation 0; out: after the chunks
    uint32_t nseq;
    const uint32_t* run_mask = nullptr;  // rows with run_mask[q] == 0 return at once (nullptr: all)
    float* v_out = nullptr;              // [nseq][n] out instead of v (nullptr: in place)
};
struct Spec2Lds {
    uint32_t v, pairs, hacc, cmin, ccnt, eh, amax;  // offsets in floats (16-byte aligned)
    size_t bytes;
};
__host__ __device__ inline uint32_t spec2_al4(uint32_t x) { return (x + 3u) & ~3u; }
__host__ __device__ inline Spec2Lds spec2_lds_layout(uint32_t n, uint32_t KL, uint32_t NP, uint32_t H) {
    // v [n + 1] | pairs float2 [n KL + NP] | hacc [H + 1] | cmin [2][H + 1] | ccnt [2][H + 2]
    // | EH [2][2][H + 1] | amax [H + 1]
    Spec2Lds L;
    uint32_t o = 0;
    L.v = o;
    o += spec2_al4(n + 1);
    L.pairs = o;
    o += spec2_al4(2 * (n * KL + NP));
    L.hacc = o;
    o += spec2_al4(H + 1);
    L.cmin = o;
    o += spec2_al4(2 * (H + 1));
    L.ccnt = o;
    o += spec2_al4(2 * (H + 2));
    L.eh = o;
    o += spec2_al4(4 * (H + 1));
    L.amax = o;
    o += spec2_al4(H + 1);
    L.bytes = (size_t)o * 4;
    return L;
}
uint32_t spec2_round_r(uint32_t R);
uint32_t spec2_round_kl(uint32_t KL);
uint32_t spec2_round_nhs(uint32_t NHS);
hipError_t launch_spec2(const Spec2Model& m, const Spec2Batch& b, hipStream_t stream);

// Time-parallel helpers (timepar.hip; Batch::run_time_parallel).  Row index tables per active
// segment r: probe run from the exact start (x; the probe from the start's light part is row
// x + xl_off), first of the segment's guess probe rows (g: the light guess, then one row per basis
// row), first of its guess end rows (e, same order), destination row (out), probe covered the
// whole segment (full: out = X), the probe's last step (pend) and the segment's (send).
struct TpRows {
    const uint32_t* x;
    const uint32_t* g;
    const uint32_t* e;
    const uint32_t* out;
    const uint32_t* full;
    const uint32_t* pend;
    const uint32_t* send;
};
// Basis rows of the guess runs (the model's heavy rows, run from unit start vectors).
struct TpBasis {
    int32_t hrow[kBandHeavy];
    uint32_t H;
};
// out[orow[r]] = in[irow[r]] (only where flag[r] != 0 when flag is given)
hipError_t launch_tp_copy_rows(const float* in, const uint32_t* irow, float* out, const uint32_t* orow,
                               uint32_t rows, uint32_t n, const uint32_t* flag, hipStream_t s);
// out rows [0, nseq): S; rows [nseq, 2 nseq): S with the basis rows at +inf (the light part).
hipError_t launch_tp_probe_starts(const float* S, float* out, uint32_t nseq, uint32_t n, const TpBasis& basis,
                                  hipStream_t s);
// flag[r] = 1: not converged; the fallback row r runs steps fbeg[r]..fend[r]-1 (none when converged)
hipError_t launch_tp_correct(const float* X, const float* G, const float* E1, const TpRows& rows, uint32_t count,
                             uint32_t xl_off, const TpBasis& basis, float* out, uint32_t n, float tol,
                             uint32_t* flag, uint32_t* fbeg, uint32_t* fend, hipStream_t s);
hipError_t launch_tp_finish(const float* S, float* scores, int64_t* best, uint32_t nseq, uint32_t n, hipStream_t s);

// v0[q][j] = fl(E[s0][j] + start[j]) for every sequence.
hipError_t launch_first_step(const CsrModel& m, const uint8_t* symbols, const uint64_t* sym_off,
                             uint32_t nseq, float* v, hipStream_t stream);

}  // namespace svh
