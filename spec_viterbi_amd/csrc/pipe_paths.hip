// Decoded paths of the pipelined latency plan (pipe.hip PATHS): the path walk.
//
// Reference semantics: the oracle's backpointer of state j at observation t is the lexicographic
// (value, row) argmin over row j's terms of GraphBLAS_impl.cpp:64-73's product
// min_k fl(fl(E[o][j] + T^T[j][k]) + v[k]) (viterbi_oracle.c step / ora_traceback; lowest row on
// ties, a term that exists with weight +inf still counts).  The kernel records, per light
// position and observation, whether F's term was taken (mask words); the heavy rows' inputs of an
// observation -- F's and S's scores and the light minimum mu -- are rebuilt where the walk needs
// them from the kernel's per-block partials (RecSrc):
//       mu(r) = min over blocks of prec[.][r+1].x   (exact: min is exact)
//       C(r)  = min over blocks of prec[.][r].y, C(0) = fl(E_S(o_0) + start_S)
//       F(r)  = F(32k) from fck, advanced by F = fl(X_FF(o_i) + F) (the kernel's speculated F,
//               exact for every row the kernel did not flag)
// The walk (one wave per sequence) is chain_paths.hip's chain_traceback_kernel -- speculative
// along light runs and heavy self-loop runs, 64 observations per round -- with the pipelined
// plan's layouts; where a heavy row's light-set term wins or ties, the lowest light position j*
// with fl(cA + v[j]) == fl(cA + mu) is recomputed from the light checkpoint below that row.
#include "pipe_common.h"

namespace svh {

using namespace dev;
using namespace pipe_dev;

namespace {

constexpr uint32_t kPTbMaxP = kPipeTbMaxP;  // light positions the j* recompute stages in LDS (x2 buffers)
constexpr uint32_t kPTbMaxN = kPTbMaxP + 2;  // states whose position map is staged in LDS

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// The heavy rows' inputs of record row r (observation r+1), rebuilt on demand from the kernel's
// per-block partials (prec[u][t] = {mu_u(t-1), C_u(t)}, u over blocks) and F's
// 32-observation checkpoints: min is exact, and F is re-advanced with the kernel's own
// fl(X_FF(o) + F).
struct RecSrc {
    const float2* prec;
    const float* fck;
    const uint8_t* sym;
    const float* hcl;  // [S][8] heavy constants (LDS)
    uint32_t len, U;
    float c0;          // C(0) = fl(E_S(o_0) + start_S)
    __device__ float F(uint32_t r) const {
        const uint32_t r0 = r & ~31u;
        float xf[31];
#pragma unroll
        for (int i = 0; i < 31; ++i) xf[i] = r0 + 1 + i <= r ? hcl[(size_t)sym[r0 + 1 + i] * 8 + 3] : 0.0f;
        float f = fck[r0 >> 5];
#pragma unroll
        for (int i = 0; i < 31; ++i)
            if (r0 + 1 + i <= r) f = xf[i] + f;
        return f;
    }
    // which = 0: mu(r) (the .x of observation r+1), 1: C(r) (the .y of observation r)
    __device__ float reduce(uint32_t t, int which) const {
        float acc = kInf;
        uint32_t u = 0;
        for (; u + 8 <= U; u += 8) {
            float x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float2 e = prec[(size_t)(u + k) * len + t];
                x[k] = which ? e.y : e.x;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc = fminf(acc, x[k]);
        }
        for (; u < U; ++u) {
            const float2 e = prec[(size_t)u * len + t];
            acc = fminf(acc, which ? e.y : e.x);
        }
        return acc;
    }
    __device__ float mu(uint32_t r) const { return reduce(r + 1, 0); }
    __device__ float C(uint32_t r) const { return r ? reduce(r, 1) : c0; }
};

// (eb, ea) of position x for symbol o in the plan's table layout: the latency plan's
// [nblk][S][SM][64] float2, or the wide plan's [nblk][S][NC][64] float4 chunks ([eb_1 .. eb_{SM-1},
// eb_0] then [ea_0 .. ea_{SM-1}], pipe_wide_kernel.h).
__device__ __forceinline__ float2 pipe_tab_pair(const PipeModel& m, uint32_t x, uint32_t o) {
    const uint32_t SM = m.SM, bsz = 64 * SM, blk = x / bsz, ln = (x % bsz) / SM, s = x % SM;
    if (!m.wide) return m.tab[(((size_t)blk * m.S + o) * SM + s) * 64 + ln];
    const float* base = reinterpret_cast<const float*>(m.tab) + ((size_t)blk * m.S + o) * pipew_chunks(SM, m.sx != 0) * 256;
    const uint32_t ib = s == 0 ? SM - 1 : s - 1, ia = SM + s;
    return make_float2(base[((ib / 4) * 64 + ln) * 4 + ib % 4], base[((ia / 4) * 64 + ln) * 4 + ia % 4]);
}

// j* of record row r for heavy row h (0 = F, 1 = S): the lowest light position p with
// fl(cA_h + v_r[p]) == fl(cA_h + mu_r), cA_h the light-set constant of h for the symbol of
// observation r+1.  v_r is recomputed by one wave from the checkpoint row c = r rounded down to
// kCkptEvery with the kernel's float operations: v_i[p] = fminf(fl(ea_p + F(i-1)),
// fl(eb_p + v_{i-1}[p-1])) (v_{i-1}[-1] = +inf), F advanced alongside from F(c).
__device__ uint32_t pipe_jstar(const PipeModel& m, const RecSrc& rs, const float* ck, uint32_t r, uint32_t h,
                               float* buf) {
    const uint32_t lane = threadIdx.x & 63u, P = m.P;
    const uint32_t c = r / kCkptEvery * kCkptEvery;
    float* cur = buf;
    float* nxt = buf + kPTbMaxP;
    const float* ckr = ck + (size_t)(c / kCkptEvery) * P;
    for (uint32_t x = lane; x < P; x += 64) cur[x] = ckr[x];
    float F = rs.F(c);
    wave_sync();
    for (uint32_t i = c + 1; i <= r; ++i) {
        const uint32_t o = rs.sym[i];
        for (uint32_t x = lane; x < P; x += 64) {
            const float2 e = pipe_tab_pair(m, x, o);
            const float pv = x ? cur[x - 1] : kInf;
            nxt[x] = fminf(e.y + F, e.x + pv);
        }
        F = rs.hcl[(size_t)o * 8 + 3] + F;  // F(i)
        wave_sync();
        float* t = cur;
        cur = nxt;
        nxt = t;
    }
    const float mu = rs.mu(r);
    const float ca = rs.hcl[(size_t)rs.sym[r + 1] * 8 + (h == 0 ? 1 : 0)];  // A_F or A_S
    const float tgt = ca + mu;
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t x = lane; x < P; x += 64)
        if (ca + cur[x] == tgt) best = min(best, x);
    for (int off = 32; off >= 1; off >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, off));
    wave_sync();  // buf is reused by the next call
    return best;
}

// One wave per sequence.  The walk is chain_paths.hip's: speculative along light runs and heavy
// self-loop runs, 64 observations per round.  Where the path is in F and F's self loop exists and
// its row is below every light row, the kernel's exact speculation check (no light term of F ever
// below its self term on a row this kernel traces) already decides F's backpointer: itself, with
// no loads; S (and F otherwise) rebuild their inputs on demand (RecSrc).
__global__ __launch_bounds__(64) void pipe_traceback_kernel(PipeModel m, FusedBatch b, const uint64_t* path_off,
                                                             int32_t* paths, const uint32_t* skip) {
    __shared__ float buf[2 * kPTbMaxP];
    // the walk's per-round lookups, staged in LDS (the masks, partials and symbols of a round's
    // 64 observations are its only global loads)
    __shared__ float hcl[32 * 8];
    __shared__ int32_t sposl[kPTbMaxN];
    __shared__ uint32_t lrowl[kPTbMaxP];
    __shared__ uint8_t pfl[kPTbMaxP];
    const uint32_t q = blockIdx.x, lane = threadIdx.x;
    if (skip && skip[q]) return;  // re-run (and traced) by the chain kernel
    for (uint32_t x = lane; x < m.S * 8; x += 64) hcl[x] = m.hc[x];
    for (uint32_t x = lane; x < m.n; x += 64) sposl[x] = m.spos[x];
    for (uint32_t x = lane; x < m.P; x += 64) {
        lrowl[x] = m.lrow[x];
        pfl[x] = m.pflags[x];
    }
    const uint32_t len = b.end[q];
    const uint32_t nblk = m.nblk, SM = m.SM, bsz = 64 * SM;
    RecSrc rs;
    rs.prec = b.prec + b.prec_off[q];
    rs.fck = b.fck + b.fck_off[q];
    rs.sym = b.symbols + b.sym_off[q];
    rs.hcl = hcl;
    rs.len = len;
    rs.U = pipe_prec_parts(m.wide != 0) * nblk;
    wave_sync();
    rs.c0 = m.rowS >= 0 ? hcl[(size_t)rs.sym[0] * 8 + 6] + m.startS : kInf;
    // F's backpointer is itself wherever the kernel's check held (see above)
    const bool f_self = ((m.hx_exist & 1u) != 0) && (!(m.hl_exist & 1u) || (uint32_t)m.rowF < lrowl[0]);

    const uint32_t* msk = b.cmask + b.cmask_off[q];
    const float* ck = b.ckpt + b.ckpt_off[q];
    const uint32_t wstride = nblk * SM * 64;
    int32_t* out = paths + path_off[q];
    const int64_t best = b.best[q];
    int32_t s = best < 0 ? -1 : (int32_t)best;
    if (lane == 0) out[len - 1] = s;
    const int hrowk[2] = {m.rowF, m.rowS};
    int64_t i = (int64_t)len - 1;  // out[i] == s is known; find out[i-1], out[i-2], ...
    while (i >= 1) {
        if (s < 0) {  // no predecessor: every earlier entry is -1 (oracle: ora_traceback)
            for (int64_t r = lane; r < i; r += 64) out[r] = -1;
            break;
        }
        const int32_t pos = sposl[s];
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
                const uint32_t pp = (uint32_t)p, blk = pp / bsz, ln = (pp % bsz) / SM, ss = pp % SM;
                const uint32_t word = msk[((uint64_t)r >> 5) * wstride + (blk * SM + ss) * 64 + ln];
                const uint32_t f = pfl[pp];
                if ((word >> (31u - ((uint32_t)r & 31u))) & 1u) {
                    pred = m.rowF;
                } else if ((f & 1u) && pp >= 1) {
                    pred = (int32_t)lrowl[pp - 1];
                    cont = true;
                }
            }
        } else if (valid && pos == -1 && f_self) {  // F's self loop (the kernel's check decided it)
            pred = m.rowF;
            cont = pred == s;
        } else if (valid) {  // heavy run: self-loops of heavy row h
            // the heavy row's lexicographic (value, row) argmin at observation r+1, re-evaluated
            // from its rebuilt inputs with the kernel's float operations: heavy terms fl(cX + vo[k])
            // and the light-set term fl(cA + mu)
            const uint32_t h = (uint32_t)(-1 - pos);
            const uint32_t rr = (uint32_t)r;
            const float* hc = hcl + (size_t)rs.sym[rr + 1] * 8;  // A_S A_F X_SS X_FF X_SF
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if ((m.hx_exist >> (h * 2 + k)) & 1u) {
                    // X[h][k]: F <- F = X_FF, S <- F = X_SF, S <- S = X_SS (F <- S never: plan)
                    const float cx = h == 0 ? hc[3] : (k == 0 ? hc[4] : hc[2]);
                    const float val = cx + (k == 0 ? rs.F(rr) : rs.C(rr));
                    const uint32_t col = (uint32_t)hrowk[k];
                    const bool take = !hex || val < hv || (val == hv && col < hcol);
                    hv = take ? val : hv;
                    hcol = take ? col : hcol;
                    hex = true;
                }
            }
            pred = hex ? (int32_t)hcol : -1;
            if ((m.hl_exist >> h) & 1u) {
                lv = hc[h == 0 ? 1 : 0] + rs.mu(rr);
                needj = !hex || !(hv < lv);  // the light set wins or ties: its lowest row j* decides
            }
            cont = !needj && pred == s;
        }
        uint64_t stop = __builtin_amdgcn_ballot_w64(!cont);
        uint32_t ls = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;  // first lane leaving the run
        while (ls < 64u && __builtin_amdgcn_readlane((int)needj, (int)ls)) {
            const uint32_t rj = (uint32_t)(i - 1 - (int64_t)ls);
            const uint32_t jp = pipe_jstar(m, rs, ck, rj, (uint32_t)(-1 - pos), buf);
            if (lane == ls) {
                const uint32_t js = jp == 0xFFFFFFFFu ? 0xFFFFFFFFu : lrowl[jp];
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

hipError_t launch_pipe_traceback(const PipeModel& m, const FusedBatch& b, const uint64_t* path_off, int32_t* paths,
                                 const uint32_t* skip, hipStream_t stream) {
    if (!b.cmask || !b.ckpt || !b.prec || !b.fck || !m.pflags || !m.spos || m.P > kPTbMaxP || m.n > kPTbMaxN ||
        m.S > 32)
        return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    hipLaunchKernelGGL(pipe_traceback_kernel, dim3(b.nseq), dim3(64), 0, stream, m, b, path_off, paths, skip);
    return hipGetLastError();
}

}  // namespace svh
