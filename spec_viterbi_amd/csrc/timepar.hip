// Time-parallel Viterbi helpers (opt-in, Batch::run_time_parallel).
//
// A long sequence is cut into segments that run concurrently from guess start vectors: a light
// guess and one unit vector per basis row (the model's heavy rows).  The segment maps are
// (min,+)-linear, so the segment's end from its exact start is the minimum of the basis runs'
// ends shifted by the start's basis scores and of the light part's run; once the light part's
// probe and the light guess's probe differ by a constant wherever the light part is not already
// dominated (tropical rank convergence within the probe length), the light guess's end plus that
// constant stands in for the light part's run.  These kernels do the check and the correction;
// the step kernels themselves are the ordinary ones.
#include "device_common.h"
#include "kernels.h"

namespace svh {

using namespace dev;

namespace {

__global__ void tp_copy_rows_kernel(const float* in, const uint32_t* irow, float* out, const uint32_t* orow,
                                    uint32_t n, const uint32_t* flag) {
    const uint32_t r = blockIdx.y;
    if (flag && !flag[r]) return;
    const float* src = in + (size_t)irow[r] * n;
    float* dst = out + (size_t)orow[r] * n;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) dst[j] = src[j];
}

__global__ void tp_probe_starts_kernel(const float* S, float* out, uint32_t nseq, uint32_t n, TpBasis basis) {
    const uint32_t r = blockIdx.y, q = r < nseq ? r : r - nseq;
    const bool light = r >= nseq;
    const float* src = S + (size_t)q * n;
    float* dst = out + (size_t)r * n;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        bool basis_row = false;
        for (uint32_t b = 0; b < basis.H; ++b) basis_row |= (uint32_t)basis.hrow[b] == j;
        dst[j] = light && basis_row ? kInf : src[j];
    }
}

// One workgroup per active segment r.  The segment's end from its exact start v is, by
// (min,+)-linearity over the split of v into its basis rows and its light part L,
//     F(v) = min( min_b F(e_b) + v_b , F(L) ).
// F(e_b) are the basis guess runs (E1 rows e+1..e+H).  F(L) is replaced by F(G) + d, G the light
// guess (E1 row e), when the probes of L (XL) and of G (GP, G row g) after the probe length agree
// up to the constant d wherever the light part can still matter: an entry of XL not below
// Y = min_b (probe of e_b) + v_b is dominated (every continuation of it is matched by the basis
// terms' at the same state), so it only has to stay dominated on the guess side too.  d is taken
// at the lowest-index minimum of the non-dominated XL entries; "agree" is within
// tol * max(1, |that minimum|).  No non-dominated entry: F(v) = the basis terms alone.  A probe
// that covered the whole segment is exact: out = X.  flag[r] = 1: not converged (the host runs
// the rest exactly from X); tol < 0 never converges.
__global__ __launch_bounds__(256) void tp_correct_kernel(const float* X, const float* G, const float* E1,
                                                         TpRows rows, uint32_t xl_off, TpBasis basis, float* out,
                                                         uint32_t n, float tol, uint32_t* flag, uint32_t* fbeg,
                                                         uint32_t* fend) {
    __shared__ float s_vh[kBandHeavy], s_v[4];
    __shared__ uint32_t s_k[4], s_ok[4];
    const uint32_t r = blockIdx.x, t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const float* x = X + (size_t)rows.x[r] * n;
    const float* xl = X + (size_t)(rows.x[r] + xl_off) * n;
    const float* g = G + (size_t)rows.g[r] * n;
    const float* e = E1 + (size_t)rows.e[r] * n;
    float* o = out + (size_t)rows.out[r] * n;
    if (rows.full[r]) {
        for (uint32_t j = t; j < n; j += 256) o[j] = x[j];
        if (t == 0) {
            flag[r] = 0;
            fbeg[r] = fend[r] = rows.pend[r];
        }
        return;
    }
    const uint32_t H = basis.H;
    if (t < H) s_vh[t] = o[basis.hrow[t]];  // the exact start's basis scores (out = S row)
    __syncthreads();
    float vh[kBandHeavy];
#pragma unroll
    for (int b = 0; b < kBandHeavy; ++b) vh[b] = (uint32_t)b < H ? s_vh[b] : kInf;
    auto dominant = [&](uint32_t j) -> float {  // Y[j]
        float y = kInf;
        for (uint32_t b = 0; b < H; ++b) y = fminf(y, g[(size_t)(b + 1) * n + j] + vh[b]);
        return y;
    };
    // pass 1: lowest-index minimum of the non-dominated light-part entries
    float bv = kInf;
    uint32_t bk = 0xFFFFFFFFu;
    for (uint32_t j = t; j < n; j += 256) {
        const float xv = xl[j];
        if (xv < dominant(j)) lex_min(bv, bk, xv, j);
    }
    for (int off = 32; off >= 1; off >>= 1) {
        const float ov = __shfl_xor(bv, off);
        const uint32_t ok = __shfl_xor(bk, off);
        lex_min(bv, bk, ov, ok);
    }
    if (lane == 0) {
        s_v[wave] = bv;
        s_k[wave] = bk;
    }
    __syncthreads();
    bv = s_v[0];
    bk = s_k[0];
    for (int w = 1; w < 4; ++w) lex_min(bv, bk, s_v[w], s_k[w]);
    const bool any_nd = bk != 0xFFFFFFFFu;
    const float d = any_nd ? xl[bk] - g[bk] : 0.0f;
    const float scale = tol * fmaxf(1.0f, fabsf(bv));
    // pass 2: agreement up to d, or dominated on both sides
    uint32_t good = tol >= 0.0f ? 1u : 0u;
    if (any_nd && good) {
        for (uint32_t j = t; j < n; j += 256) {
            const float xv = xl[j], gv = g[j], y = dominant(j);
            const bool both_inf = __builtin_isinf(xv) && __builtin_isinf(gv);
            const bool agree = fabsf(xv - gv - d) <= scale;
            const bool dom = xv >= y && gv + d >= y;
            good &= (both_inf || agree || dom) ? 1u : 0u;
        }
    }
    for (int off = 32; off >= 1; off >>= 1) good &= (uint32_t)__shfl_xor((int)good, off);
    if (lane == 0) s_ok[wave] = good;
    __syncthreads();
    const bool converged = s_ok[0] && s_ok[1] && s_ok[2] && s_ok[3];
    if (converged) {
        for (uint32_t j = t; j < n; j += 256) {
            float v = any_nd ? e[j] + d : kInf;
            for (uint32_t b = 0; b < H; ++b) v = fminf(v, e[(size_t)(b + 1) * n + j] + vh[b]);
            o[j] = v;
        }
    }
    if (t == 0) {
        flag[r] = converged ? 0u : 1u;
        fbeg[r] = rows.pend[r];
        fend[r] = converged ? rows.pend[r] : rows.send[r];
    }
}

// scores[q] = S[q], best[q] = lowest-index argmin (as the step kernels' epilogues)
__global__ __launch_bounds__(256) void tp_finish_kernel(const float* S, float* scores, int64_t* best, uint32_t n) {
    __shared__ float s_v[4];
    __shared__ uint32_t s_k[4];
    const uint32_t q = blockIdx.x, t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const float* src = S + (size_t)q * n;
    float* dst = scores + (size_t)q * n;
    float bv = kInf;
    uint32_t bk = 0xFFFFFFFFu;
    for (uint32_t j = t; j < n; j += 256) {
        const float v = src[j];
        dst[j] = v;
        lex_min(bv, bk, v, j);
    }
    for (int off = 32; off >= 1; off >>= 1) {
        const float ov = __shfl_xor(bv, off);
        const uint32_t ok = __shfl_xor(bk, off);
        lex_min(bv, bk, ov, ok);
    }
    if (lane == 0) {
        s_v[wave] = bv;
        s_k[wave] = bk;
    }
    __syncthreads();
    if (t == 0) {
        bv = s_v[0];
        bk = s_k[0];
        for (int w = 1; w < 4; ++w) lex_min(bv, bk, s_v[w], s_k[w]);
        best[q] = bk == 0xFFFFFFFFu ? -1 : (int64_t)bk;
    }
}

}  // namespace

hipError_t launch_tp_copy_rows(const float* in, const uint32_t* irow, float* out, const uint32_t* orow,
                               uint32_t rows, uint32_t n, const uint32_t* flag, hipStream_t s) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(tp_copy_rows_kernel, dim3((n + 255) / 256, rows), dim3(256), 0, s, in, irow, out, orow, n,
                       flag);
    return hipGetLastError();
}

hipError_t launch_tp_probe_starts(const float* S, float* out, uint32_t nseq, uint32_t n, const TpBasis& basis,
                                  hipStream_t s) {
    if (nseq == 0) return hipSuccess;
    if (basis.H > (uint32_t)kBandHeavy) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tp_probe_starts_kernel, dim3((n + 255) / 256, 2 * nseq), dim3(256), 0, s, S, out, nseq, n,
                       basis);
    return hipGetLastError();
}

hipError_t launch_tp_correct(const float* X, const float* G, const float* E1, const TpRows& rows, uint32_t count,
                             uint32_t xl_off, const TpBasis& basis, float* out, uint32_t n, float tol,
                             uint32_t* flag, uint32_t* fbeg, uint32_t* fend, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (basis.H > (uint32_t)kBandHeavy) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tp_correct_kernel, dim3(count), dim3(256), 0, s, X, G, E1, rows, xl_off, basis, out, n, tol,
                       flag, fbeg, fend);
    return hipGetLastError();
}

hipError_t launch_tp_finish(const float* S, float* scores, int64_t* best, uint32_t nseq, uint32_t n, hipStream_t s) {
    if (nseq == 0) return hipSuccess;
    hipLaunchKernelGGL(tp_finish_kernel, dim3(nseq), dim3(256), 0, s, S, scores, best, n);
    return hipGetLastError();
}

}  // namespace svh
