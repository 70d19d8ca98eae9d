// Time-parallel Viterbi helpers (opt-in, Batch::run_time_parallel).
//
// A long sequence is cut into segments that run concurrently from a guess start vector; the
// segment maps are (min,+)-linear, F(v + c) = F(v) + c, so once a segment's run from the exact
// start and its run from the guess differ by a constant (tropical rank convergence within the
// probe length), the guess run's end plus that constant is the segment's end.  These kernels do
// the check and the correction; the step kernels themselves are the ordinary ones.
#include "device_common.h"
#include "kernels.h"

namespace svh {

using namespace dev;

namespace {

__global__ void tp_copy_rows_kernel(const float* in, const uint32_t* irow, float* out, const uint32_t* orow,
                                    uint32_t n) {
    const uint32_t r = blockIdx.y;
    const float* src = in + (size_t)irow[r] * n;
    float* dst = out + (size_t)orow[r] * n;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) dst[j] = src[j];
}

// One workgroup per active segment r.  X: the probe run from the exact start, G: the probe run from
// the guess (same observations), E1: the guess run's segment end.  Converged when both runs have
// the same +inf pattern and X - G spans at most tol * |best X|: out = E1 + d, d = X - G at the lowest-index
// argmin of X (the state a best path runs through).  A probe that covered the whole segment is
// exact: out = X.  flag[r] = 1 when not converged (the host then runs the rest exactly).
__global__ __launch_bounds__(256) void tp_correct_kernel(const float* X, const float* G, const float* E1,
                                                         TpRows rows, float* out, uint32_t n, float tol,
                                                         uint32_t* flag) {
    __shared__ float s_min[4], s_max[4], s_v[4], s_d[4];
    __shared__ uint32_t s_k[4], s_mis[4];
    const uint32_t r = blockIdx.x, t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const float* x = X + (size_t)rows.x[r] * n;
    const float* g = G + (size_t)rows.g[r] * n;
    const float* e = E1 + (size_t)rows.e[r] * n;
    float* o = out + (size_t)rows.out[r] * n;
    if (rows.full[r]) {
        for (uint32_t j = t; j < n; j += 256) o[j] = x[j];
        if (t == 0) flag[r] = 0;
        return;
    }
    float dmin = kInf, dmax = -kInf, bv = kInf, bd = 0.0f;
    uint32_t bk = 0xFFFFFFFFu, mis = 0;
    for (uint32_t j = t; j < n; j += 256) {
        const float xv = x[j], gv = g[j];
        const bool xi = __builtin_isinf(xv), gi = __builtin_isinf(gv);
        mis |= (xi != gi) ? 1u : 0u;
        if (!xi && !gi) {
            const float d = xv - gv;
            dmin = fminf(dmin, d);
            dmax = fmaxf(dmax, d);
            if (xv < bv || (xv == bv && j < bk)) {
                bv = xv;
                bk = j;
                bd = d;
            }
        }
    }
    for (int off = 32; off >= 1; off >>= 1) {
        dmin = fminf(dmin, __shfl_xor(dmin, off));
        dmax = fmaxf(dmax, __shfl_xor(dmax, off));
        mis |= __shfl_xor(mis, off);
        const float ov = __shfl_xor(bv, off), od = __shfl_xor(bd, off);
        const uint32_t ok = __shfl_xor(bk, off);
        if (ov < bv || (ov == bv && ok < bk)) {
            bv = ov;
            bk = ok;
            bd = od;
        }
    }
    if (lane == 0) {
        s_min[wave] = dmin;
        s_max[wave] = dmax;
        s_v[wave] = bv;
        s_d[wave] = bd;
        s_k[wave] = bk;
        s_mis[wave] = mis;
    }
    __syncthreads();
    dmin = s_min[0];
    dmax = s_max[0];
    bv = s_v[0];
    bd = s_d[0];
    bk = s_k[0];
    mis = s_mis[0];
    for (int w = 1; w < 4; ++w) {
        dmin = fminf(dmin, s_min[w]);
        dmax = fmaxf(dmax, s_max[w]);
        mis |= s_mis[w];
        if (s_v[w] < bv || (s_v[w] == bv && s_k[w] < bk)) {
            bv = s_v[w];
            bk = s_k[w];
            bd = s_d[w];
        }
    }
    // tol is relative to the best score's magnitude (the rounding noise of X - G scales with it)
    const bool converged = !mis && (bk == 0xFFFFFFFFu || dmax - dmin <= tol * fmaxf(1.0f, fabsf(bv)));
    if (converged) {
        const float d = bk == 0xFFFFFFFFu ? 0.0f : bd;
        for (uint32_t j = t; j < n; j += 256) o[j] = e[j] + d;
    }
    if (t == 0) flag[r] = converged ? 0u : 1u;
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
                               uint32_t rows, uint32_t n, hipStream_t s) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(tp_copy_rows_kernel, dim3((n + 255) / 256, rows), dim3(256), 0, s, in, irow, out, orow, n);
    return hipGetLastError();
}

hipError_t launch_tp_correct(const float* X, const float* G, const float* E1, const TpRows& rows, uint32_t count,
                             float* out, uint32_t n, float tol, uint32_t* flag, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(tp_correct_kernel, dim3(count), dim3(256), 0, s, X, G, E1, rows, out, n, tol, flag);
    return hipGetLastError();
}

hipError_t launch_tp_finish(const float* S, float* scores, int64_t* best, uint32_t nseq, uint32_t n, hipStream_t s) {
    if (nseq == 0) return hipSuccess;
    hipLaunchKernelGGL(tp_finish_kernel, dim3(nseq), dim3(256), 0, s, S, scores, best, n);
    return hipGetLastError();
}

}  // namespace svh
