// Generic fallback step kernel, path traceback, _spec precompute/run kernels and launchers.
#include "device_common.h"
#include "kernels.h"

namespace svh {

using namespace dev;

namespace {

// --------------------------------------------------------------------------------------------
// Generic fallback (any in-degree distribution, n up to the LDS capacity): one workgroup per
// sequence, thread-strided rows, CSR terms read from global memory (L1/L2 resident).
// Same association as the fused kernel (GraphBLAS_impl.cpp:64-73).
// --------------------------------------------------------------------------------------------
template <bool PATHS>
__global__ __launch_bounds__(1024) void generic_viterbi_kernel(CsrModel m, FusedBatch b) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t n = m.n, B = blockDim.x, t = threadIdx.x, q = blockIdx.x;
    const uint32_t lane = t & 63u, wave = t >> 6;
    const uint32_t vstride = align4(n);
    float* vb0 = lds;
    float* vb1 = lds + vstride;
    float* red = lds + 2 * vstride;
    const uint8_t* sym = b.symbols + b.sym_off[q];
    const uint32_t len = b.end[q];
    uint32_t i0 = b.begin[q];
    if (i0 == 0) {
        const float* e0 = m.emis + (size_t)sym[0] * n;
        for (uint32_t j = t; j < n; j += B) vb0[j] = e0[j] + m.start[j];
        i0 = 1;
    } else {
        const float* vin = b.v_in + (size_t)b.v_in_row[q] * n;
        for (uint32_t j = t; j < n; j += B) vb0[j] = vin[j];
    }
    __syncthreads();
    uint16_t* bp = PATHS ? b.bp + b.bp_off[q] : nullptr;
    uint32_t cur = 0;
    for (uint32_t i = i0; i < len; ++i) {
        const float* e = m.emis + (size_t)sym[i] * n;
        const float* vc = cur ? vb1 : vb0;
        float* vn = cur ? vb0 : vb1;
        for (uint32_t j = t; j < n; j += B) {
            const float ej = e[j];
            float r = kInf;
            uint32_t rk = 0xFFFFFFFFu;
            for (uint32_t p = m.rowptr[j]; p < m.rowptr[j + 1]; ++p) {
                const float term = (ej + m.val[p]) + vc[m.col[p]];
                if constexpr (PATHS) lex_min(r, rk, term, m.col[p]);
                else r = fminf(r, term);
            }
            vn[j] = r;
            if constexpr (PATHS) bp[(size_t)(i - 1) * n + j] = (uint16_t)(rk == 0xFFFFFFFFu ? kNoPred : rk);
        }
        __syncthreads();
        cur ^= 1u;
    }
    const float* vc = cur ? vb1 : vb0;
    float* out = b.scores + (size_t)q * n;
    float bv = kInf;
    uint32_t bk = 0xFFFFFFFFu;
    for (uint32_t j = t; j < n; j += B) {
        out[j] = vc[j];
        lex_min(bv, bk, vc[j], j);
    }
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

// --------------------------------------------------------------------------------------------
// Path traceback: one workgroup per sequence stages blocks of backpointer rows in LDS with
// coalesced loads, then one lane walks the block.
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void traceback_kernel(FusedBatch b, const uint64_t* path_off,
                                                        int32_t* paths, uint32_t n,
                                                        uint32_t rows_per_block) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tb_lds[];
    uint32_t* state = tb_lds;
    uint16_t* sbp = reinterpret_cast<uint16_t*>(tb_lds + 4);
    const uint32_t q = blockIdx.x, t = threadIdx.x;
    const uint32_t len = b.end[q];
    const uint16_t* bp = b.bp + b.bp_off[q];
    int32_t* out = paths + path_off[q];
    if (t == 0) {
        const int64_t s = b.best[q];
        state[0] = s < 0 ? kNoPred : (uint32_t)s;
        out[len - 1] = s < 0 ? -1 : (int32_t)s;
    }
    __syncthreads();
    for (int64_t hi = (int64_t)len - 1; hi >= 1;) {
        const int64_t lo = hi - (int64_t)rows_per_block > 0 ? hi - (int64_t)rows_per_block : 0;
        const uint32_t blk = (uint32_t)(hi - lo);  // rows lo .. hi-1 hold steps lo+1 .. hi
        const uint16_t* src = bp + (size_t)lo * n;
        const size_t cnt = (size_t)blk * n;
        for (size_t x = t; x < cnt; x += blockDim.x) sbp[x] = src[x];
        __syncthreads();
        if (t == 0) {
            uint32_t s = state[0];
            for (int64_t r = hi; r > lo; --r) {
                s = (s == kNoPred) ? kNoPred : sbp[(size_t)(r - 1 - lo) * n + s];
                out[r - 1] = (s == kNoPred) ? -1 : (int32_t)s;
            }
            state[0] = s;
        }
        __syncthreads();
        hi = lo;
    }
}

// --------------------------------------------------------------------------------------------
// _spec precompute and run kernels (reference: GraphBLAS_spec_impl.cpp:15-36, 50-97, 146-181).
// --------------------------------------------------------------------------------------------
__global__ void spec_fold_kernel(CsrModel m, float* mfold) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = (uint64_t)m.nnz * m.S;
    if (x >= total) return;
    const uint32_t p = (uint32_t)(x / m.S), i = (uint32_t)(x % m.S);
    mfold[x] = m.emis[(size_t)i * m.n + m.row_of[p]] + m.val[p];  // diag(E_i) (x) T^T
}

__global__ void spec_scatter_kernel(CsrModel m, const float* mfold, float* h1, uint32_t pstride) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = (uint64_t)m.nnz * m.S;
    if (x >= total) return;
    const uint32_t p = (uint32_t)(x / m.S), o = (uint32_t)(x % m.S);
    h1[((size_t)o * m.n + m.row_of[p]) * pstride + m.col[p]] = mfold[x];
}

// K3: grid (m-tiles of 256, row j, kp * nsc + sc); one output column per thread, the <= 32
// symbols of chunk sc in registers; M_i[j][p] is wave-uniform (scalar loads).  Four p's in
// flight per iteration.
constexpr int kExtSym = 32;
__global__ __launch_bounds__(256) void spec_extend_kernel(CsrModel m, const float* mfold,
                                                          const float* h_prev, float* h_new,
                                                          uint32_t pstride, uint32_t nsc) {
    const uint32_t mcol = blockIdx.x * 256 + threadIdx.x;
    const uint32_t j = blockIdx.y;
    const uint32_t kp = blockIdx.z / nsc, sc = blockIdx.z % nsc;
    const uint32_t S = m.S, n = m.n;
    const uint32_t i0 = sc * kExtSym;
    const uint32_t ni = min((uint32_t)kExtSym, S - i0);
    const bool live = mcol < n;
    float acc[kExtSym];
#pragma unroll
    for (int i = 0; i < kExtSym; ++i) acc[i] = kInf;
    const float* hp = h_prev + (size_t)kp * n * pstride + (live ? mcol : 0);
    const uint32_t pb = m.rowptr[j], pe = m.rowptr[j + 1];
    for (uint32_t p = pb; p < pe; ++p) {
        const float hv = hp[(size_t)m.col[p] * pstride];
        const float* mf = mfold + (size_t)p * S + i0;
#pragma unroll
        for (int i = 0; i < kExtSym; ++i)
            if ((uint32_t)i < ni) acc[i] = fminf(acc[i], mf[i] + hv);  // fl(M_i[j][p] + H[p][m])
    }
    if (mcol < pstride) {
#pragma unroll
        for (int i = 0; i < kExtSym; ++i)
            if ((uint32_t)i < ni)
                h_new[(((size_t)kp * S + i0 + i) * n + j) * pstride + mcol] = live ? acc[i] : kInf;
    }
}

// K4: one level-L chunk, dense (min,+) GEMV per sequence: v'[j] = min_m fl(H[key][j][m] + v[m]).
// grid (row blocks of 16, nseq), 256 threads = 4 waves x 4 rows, float4 loads along the row.
// One level-L chunk: v_dst[q][j] = min_m fl(H_key[j][m] + v_src[q][m]) (GraphBLAS_spec_impl.cpp:76).
// HBM-bound: every sequence streams one dense n x pstride product per chunk.  A workgroup takes
// kChunkRows rows (kChunkRowsPerWave per wave, interleaved so each lane keeps that many 16-byte
// loads in flight) against v staged once in LDS; the product rows are read non-temporally (a
// product is reused only at a random later chunk, long after L2 would have dropped it).
constexpr int kChunkRowsPerWave = 8;
constexpr int kChunkRows = 4 * kChunkRowsPerWave;
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void spec_chunk_kernel(CsrModel m, const float* products,
                                                         SpecChunkBatch c, uint32_t pstride) {
    extern __shared__ __attribute__((aligned(16))) float sv[];
    const uint32_t q = blockIdx.y;
    if (c.chunk >= c.nchunks[q]) return;
    const uint32_t n = m.n, t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const float* vsrc = c.v_src + (size_t)q * n;
    for (uint32_t x = t; x < pstride; x += 256) sv[x] = x < n ? vsrc[x] : kInf;
    const uint8_t* sym = c.symbols + c.sym_off[q] + 1 + (size_t)c.chunk * c.level;
    uint64_t key = 0;
    for (uint32_t r = 0; r < c.level; ++r) key = key * m.S + sym[r];
    __syncthreads();
    const float* Hk = products + key * (size_t)n * pstride;
    const uint32_t nvec = pstride / 4;
    const float4* v4 = reinterpret_cast<const float4*>(sv);
    const uint32_t j0 = blockIdx.x * kChunkRows + wave * kChunkRowsPerWave;
    const f32x4* rows[kChunkRowsPerWave];
    float acc[kChunkRowsPerWave];
#pragma unroll
    for (int r = 0; r < kChunkRowsPerWave; ++r) {
        const uint32_t j = min(j0 + r, n - 1);  // rows past n repeat the last one (result dropped)
        rows[r] = reinterpret_cast<const f32x4*>(Hk + (size_t)j * pstride);
        acc[r] = kInf;
    }
    for (uint32_t x = lane; x < nvec; x += 64) {
        f32x4 h[kChunkRowsPerWave];
#pragma unroll
        for (int r = 0; r < kChunkRowsPerWave; ++r) h[r] = __builtin_nontemporal_load(rows[r] + x);
        const float4 v = v4[x];
#pragma unroll
        for (int r = 0; r < kChunkRowsPerWave; ++r)
            acc[r] = fminf(acc[r], fminf(fminf(h[r].x + v.x, h[r].y + v.y), fminf(h[r].z + v.z, h[r].w + v.w)));
    }
#pragma unroll
    for (int r = 0; r < kChunkRowsPerWave; r += 2) wave_min63x2(acc[r], acc[r + 1]);
    if (lane == 63) {
#pragma unroll
        for (int r = 0; r < kChunkRowsPerWave; ++r)
            if (j0 + r < n) c.v_dst[(size_t)q * n + j0 + r] = acc[r];
    }
}

__global__ void first_step_kernel(CsrModel m, const uint8_t* symbols, const uint64_t* sym_off,
                                  float* v) {
    const uint32_t q = blockIdx.y;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m.n) return;
    const uint32_t o = symbols[sym_off[q]];
    v[(size_t)q * m.n + j] = m.emis[(size_t)o * m.n + j] + m.start[j];
}

hipError_t set_lds_limit(const void* fn, size_t bytes) {
    if (bytes <= 64 * 1024) return hipSuccess;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

int family_rmax(int fam) {
    static const int r[kNumFamilies] = {2, 2, 4, 8, 16};
    return (fam >= 0 && fam < kNumFamilies) ? r[fam] : 0;
}
int family_hmax(int fam) {
    static const int h[kNumFamilies] = {2, 2, 4, 4, 4};
    return (fam >= 0 && fam < kNumFamilies) ? h[fam] : 0;
}
int family_xmax(int fam) {
    static const int x[kNumFamilies] = {2, 2, 4, 4, 4};
    return (fam >= 0 && fam < kNumFamilies) ? x[fam] : 0;
}
int family_mode(int fam) { return fam == kFamR2Uni ? kHeavyUniform : kHeavyGeneral; }

hipError_t launch_fused(const FusedModel& m, const FusedBatch& b, int fam, bool paths,
                        hipStream_t stream) {
    const void* fn = nullptr;
    switch (fam) {
        case kFamR2Uni: fn = fused_kernel_r2uni((int)m.slots, paths); break;
        case kFamR2: fn = fused_kernel_r2((int)m.slots, paths); break;
        case kFamR4: fn = fused_kernel_r4((int)m.slots, paths); break;
        case kFamR8: fn = fused_kernel_r8((int)m.slots, paths); break;
        case kFamR16: fn = fused_kernel_r16((int)m.slots, paths); break;
        default: break;
    }
    if (!fn) return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    const size_t lds = fused_lds_bytes(m);
    hipError_t e = set_lds_limit(fn, lds);
    if (e != hipSuccess) return e;
    FusedModel mm = m;
    FusedBatch bb = b;
    void* args[] = {&mm, &bb};
    return hipLaunchKernel(fn, dim3(b.nseq), dim3(m.B), args, lds, stream);
}

size_t generic_lds_bytes(uint32_t n) {
    return (2 * (size_t)((n + 3) & ~3u) + 2 * kMaxWaves) * sizeof(float);
}

hipError_t launch_generic(const CsrModel& m, const FusedBatch& b, int threads, bool paths,
                          hipStream_t stream) {
    const void* fn = paths ? reinterpret_cast<const void*>(&generic_viterbi_kernel<true>)
                           : reinterpret_cast<const void*>(&generic_viterbi_kernel<false>);
    if (b.nseq == 0) return hipSuccess;
    const size_t lds = generic_lds_bytes(m.n);
    hipError_t e = set_lds_limit(fn, lds);
    if (e != hipSuccess) return e;
    CsrModel mm = m;
    FusedBatch bb = b;
    void* args[] = {&mm, &bb};
    return hipLaunchKernel(fn, dim3(b.nseq), dim3(threads), args, lds, stream);
}

hipError_t launch_traceback(const FusedBatch& b, const uint64_t* path_off, int32_t* paths,
                            uint32_t n, hipStream_t stream) {
    if (b.nseq == 0) return hipSuccess;
    uint32_t rows = (uint32_t)((64 * 1024) / (2 * (size_t)n));
    if (rows < 1) rows = 1;
    const size_t lds = 16 + (size_t)rows * n * sizeof(uint16_t);
    const void* fn = reinterpret_cast<const void*>(&traceback_kernel);
    hipError_t e = set_lds_limit(fn, lds);
    if (e != hipSuccess) return e;
    FusedBatch bb = b;
    const uint64_t* po = path_off;
    int32_t* pp = paths;
    uint32_t nn = n;
    void* args[] = {&bb, &po, &pp, &nn, &rows};
    return hipLaunchKernel(fn, dim3(b.nseq), dim3(256), args, lds, stream);
}

hipError_t launch_spec_fold(const CsrModel& m, float* mfold, hipStream_t stream) {
    const uint64_t total = (uint64_t)m.nnz * m.S;
    if (total == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)((total + 255) / 256);
    hipLaunchKernelGGL(spec_fold_kernel, dim3(blocks), dim3(256), 0, stream, m, mfold);
    return hipGetLastError();
}

hipError_t launch_spec_densify(const CsrModel& m, const float* mfold, float* h1, uint32_t pstride,
                               hipStream_t stream) {
    const size_t words = (size_t)m.S * m.n * pstride;
    hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(h1), 0x7f800000, words, stream);
    if (e != hipSuccess) return e;
    const uint64_t total = (uint64_t)m.nnz * m.S;
    if (total == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)((total + 255) / 256);
    hipLaunchKernelGGL(spec_scatter_kernel, dim3(blocks), dim3(256), 0, stream, m, mfold, h1,
                       pstride);
    return hipGetLastError();
}

hipError_t launch_spec_extend(const CsrModel& m, const float* mfold, const float* h_prev,
                              uint64_t kprev, float* h_new, uint32_t pstride, hipStream_t stream) {
    const uint32_t nsc = (m.S + kExtSym - 1) / kExtSym;
    const uint64_t gz = kprev * nsc;
    if (gz == 0) return hipSuccess;
    if (gz > 65535 || m.n > 65535) return hipErrorInvalidValue;
    dim3 grid((pstride + 255) / 256, m.n, (uint32_t)gz);
    hipLaunchKernelGGL(spec_extend_kernel, grid, dim3(256), 0, stream, m, mfold, h_prev, h_new,
                       pstride, nsc);
    return hipGetLastError();
}

hipError_t launch_spec_chunk(const CsrModel& m, const float* products, const SpecChunkBatch& c,
                             uint32_t pstride, hipStream_t stream) {
    if (c.nseq == 0) return hipSuccess;
    dim3 grid((m.n + kChunkRows - 1) / kChunkRows, c.nseq);
    const size_t lds = (size_t)pstride * sizeof(float);
    const void* fn = reinterpret_cast<const void*>(&spec_chunk_kernel);
    hipError_t e = set_lds_limit(fn, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(spec_chunk_kernel, grid, dim3(256), lds, stream, m, products, c, pstride);
    return hipGetLastError();
}

hipError_t launch_first_step(const CsrModel& m, const uint8_t* symbols, const uint64_t* sym_off,
                             uint32_t nseq, float* v, hipStream_t stream) {
    if (nseq == 0) return hipSuccess;
    dim3 grid((m.n + 255) / 256, nseq);
    hipLaunchKernelGGL(first_step_kernel, grid, dim3(256), 0, stream, m, symbols, sym_off, v);
    return hipGetLastError();
}

}  // namespace svh
