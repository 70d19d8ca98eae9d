// Chain ("band") Viterbi step kernel (gfx950) for the MSV model shape of the reference's .chmm
// files (chmm_files/silent_hmm_to_chmm.py: N, M_1..M_L, C): every light row M_j has terms only
// from the heavy row N and from M_{j-1}; the heavy rows N and C take one shared weight from every
// M_j plus a self loop.
//
// Reference hot loop: Viterbi_impl/GraphBLAS_impl.cpp:59-73 (same association, bit-identical):
//     v'[j] = min_k fl( fl(E[o][j] + T^T[j][k]) + v[k] )
//
// One workgroup walks every observation of one sequence, one barrier per observation.
//   * Light scores never leave VGPRs: position p = t*SM + s is slot s of thread t, so the chain
//     predecessor of slot s > 0 is the thread's own slot s-1; slot 0 takes lane-1's last slot by
//     one DPP wave_shr:1, and lane 0 takes the previous wave's last value from a 1-float LDS
//     boundary slot.
//   * Heavy rows use min_{k in U} fl(a + v[k]) == fl(a + min_{k in U} v[k]) (fp32 add is
//     monotone), U = all light rows: each wave reduces min over its slots by DPP and publishes
//     one partial per observation; every thread then recomputes the heavy scores redundantly from
//     the partials, so they live in VGPRs too.  The reduction of observation i feeds the heavy
//     scores of observation i+1, which the light rows read at i+2: it is off the light chain.
//   * Emission rows (pre-permuted to the lane-consecutive slot layout, with the folded heavy
//     constants fl(E_h + w) as a tail) stream into a 3-slot LDS ring by LDS-DMA, two
//     observations ahead, counted vmcnt across the raw s_barrier.
#include "device_common.h"
#include "kernels.h"

namespace svh {

using namespace dev;

namespace {

// wave_shr:1 -- lane l receives lane l-1's value; lane 0 keeps `old`.
__device__ __forceinline__ float wave_shr1(float x, float old) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                                  __builtin_bit_cast(int, x), 0x138,
                                                                  0xf, 0xf, false));
}

// Retire all but the `k` most recent vector-memory ops of this wave, drain LDS, barrier.
__device__ __forceinline__ void wait_keep_barrier(uint32_t k) {
    switch (k) {
#define SVH_W(K)                                                                             \
    case K:                                                                                  \
        asm volatile("s_waitcnt vmcnt(" #K ")\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
        break;
        SVH_W(0) SVH_W(1) SVH_W(2) SVH_W(3) SVH_W(4) SVH_W(5) SVH_W(6) SVH_W(7)
#undef SVH_W
        default:
            asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

// Diagnostic cycle stamp (STAMP builds only): s_memtime, drained, fenced from rescheduling.
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long x;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(x)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return x;
}

template <int SM, int HA, bool STAMP = false>
__global__ __launch_bounds__(kMaxBandThreads) void band_viterbi_kernel(BandModel m, FusedBatch b) {
    constexpr int HM = kBandHeavy;
    extern __shared__ __attribute__((aligned(16))) float lds[];

    const uint32_t B = m.B, n = m.n, erow = m.erow, W = B >> 6;
    const uint32_t t = threadIdx.x, lane = t & 63u, q = blockIdx.x;
    if (b.run_mask && b.run_mask[q] == 0) return;  // fallback pass: only the marked rows
    const uint32_t wave = (uint32_t)uniform((int)(t >> 6));  // wave-uniform: scalar DMA loop and waits
    const uint32_t tail = SM * B;
    const float* __restrict__ erows = m.erows;

    // LDS: ering[3][erow] | part[2][kMaxWaves] | bnd[2][kMaxWaves] | red[2][kMaxWaves] | symbols
    float* ering = lds;
    float* part = lds + 3 * erow;
    float* bnd = part + 2 * kMaxWaves;
    float* red = bnd + 2 * kMaxWaves;
    uint32_t* symr = reinterpret_cast<uint32_t*>(red + 2 * kMaxWaves);

    // loop-invariant weights and the exception map in registers
    float aw[HA][SM], bw[SM];
#pragma unroll
    for (int s = 0; s < SM; ++s) {
        bw[s] = m.bw[s * B + t];
#pragma unroll
        for (int h = 0; h < HA; ++h) aw[h][s] = m.aw[(size_t)h * tail + s * B + t];
    }
    // ---- sequence setup (same symbol staging as the fused kernel) -------------------------
    const uint8_t* sym = b.symbols + b.sym_off[q];
    const uint32_t len = b.end[q];
    uint32_t i = b.begin[q];
    const bool fresh = (i == 0);
    uint32_t sbase = fresh ? 0u : (i & ~3u);
    auto stage_symbols = [&](uint32_t from) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(sym + from);
        const uint32_t avail = (len + kSymPad - from) / 4;
        const uint32_t words = min((uint32_t)(kSymChunk + 64) / 4, avail);
        for (uint32_t x = t; x < words; x += B) symr[x] = src[x];
    };
    stage_symbols(sbase);
    auto sym_at = [&](uint32_t idx) -> uint32_t {
        return reinterpret_cast<const uint8_t*>(symr)[idx - sbase];
    };
    // This wave's share of one emission row: 1 KiB chunks wave, wave+W, ...
    const uint32_t chunks = erow >> 8;
    const uint32_t kdma = wave < chunks ? (chunks - wave + W - 1) / W : 0u;
    auto dma_row = [&](uint32_t o, float* slot) {
        const float* row = erows + (size_t)o * erow;
        for (uint32_t c = wave; c < chunks; c += W)
            lds_dma16(row + c * 256u + lane * 4u, uniform(lds_addr(slot + c * 256u)));
    };

    // ---- initial scores ----------------------------------------------------------------------
    float v[SM], vh[HM];
    if (fresh) {
        const float* e0 = erows + (size_t)sym[0] * erow;
#pragma unroll
        for (int s = 0; s < SM; ++s) v[s] = e0[s * B + t] + m.start[s * B + t];  // diag(E[s0]) (x) start
#pragma unroll
        for (int h = 0; h < HM; ++h) vh[h] = m.hvalid[h] ? e0[tail + kBandTailE + h] + m.hstart[h] : kInf;
        i = 1;
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
    // publish partial / boundary of the initial scores under parity (i-1)&1
    {
        const uint32_t par = (i - 1) & 1u;
        if (t < 4u * kMaxWaves) part[t] = kInf;  // both parities, waves >= W stay +inf
        __syncthreads();
        float pm = v[0];
#pragma unroll
        for (int s = 1; s < SM; ++s) pm = fminf(pm, v[s]);
        pm = wave_min63(pm);
        if (lane == 63) {
            part[par * kMaxWaves + wave] = pm;
            bnd[par * kMaxWaves + wave] = v[SM - 1];
        }
    }
    __syncthreads();  // symbols staged, partials published
    if (i < len) {
        dma_row(uniform(sym_at(i)), ering);
        dma_row(uniform(sym_at(i + 1)), ering + erow);  // zero padding past len: symbol 0
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

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

    // ---- one observation -------------------------------------------------------------------
    auto step = [&](const float* ecur, float* enext2) {
        mark(0);  // barrier wait + loop control
        if (i + 3 >= sbase + kSymChunk) {  // uniform: refill the symbol ring (rare)
            sbase = i & ~3u;
            __syncthreads();
            stage_symbols(sbase);
            __syncthreads();
        }
        const uint32_t o2 = sym_at(i + 2);
        const uint32_t rp = ((i - 1) & 1u) * kMaxWaves, wp = (i & 1u) * kMaxWaves;

        // LDS reads: own emissions, folded heavy constants, wave partials, boundary
        float e[SM];
#pragma unroll
        for (int s = 0; s < SM; ++s) e[s] = ecur[s * B + t];
        const float4 c0 = *reinterpret_cast<const float4*>(ecur + tail);
        const float4 c1 = *reinterpret_cast<const float4*>(ecur + tail + 4);
        float4 pq[kMaxWaves / 4];
#pragma unroll
        for (int x = 0; x < kMaxWaves / 4; ++x) pq[x] = *reinterpret_cast<const float4*>(part + rp + 4 * x);
        const float bv = wave ? bnd[rp + wave - 1] : kInf;
        mark(1);  // LDS reads issued and landed

        // heavy rows from the partials of the previous observation
        float mu = kInf;
#pragma unroll
        for (int x = 0; x < kMaxWaves / 4; ++x)
            mu = fminf(mu, fminf(fminf(pq[x].x, pq[x].y), fminf(pq[x].z, pq[x].w)));
        const float cst[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        float vhn[HM];
#pragma unroll
        for (int h = 0; h < HM; ++h) {
            float a = cst[kBandTailA + h] + mu;
#pragma unroll
            for (int k = 0; k < HM; ++k) a = fminf(a, cst[band_tail_x(h, k)] + vh[k]);
            vhn[h] = a;
        }

        // light rows: emission masking fused with the two-term (min,+) product
        const float p0 = wave_shr1(v[SM - 1], bv);
        float vn[SM];
#pragma unroll
        for (int s = 0; s < SM; ++s) {
            const float pv = s == 0 ? p0 : v[s - 1];
            float r = (e[s] + bw[s]) + pv;
#pragma unroll
            for (int h = 0; h < HA; ++h) r = fminf(r, (e[s] + aw[h][s]) + vh[h]);
            vn[s] = r;
        }
        mark(2);  // heavy + light updates
        float pm = vn[0];
#pragma unroll
        for (int s = 1; s < SM; ++s) pm = fminf(pm, vn[s]);
        pm = wave_min63(pm);
        mark(3);  // partial reduction
        if (lane == 63) {
            part[wp + wave] = pm;
            bnd[wp + wave] = vn[SM - 1];
        }
        mark(4);  // LDS writes drained
#pragma unroll
        for (int s = 0; s < SM; ++s) v[s] = vn[s];
#pragma unroll
        for (int h = 0; h < HM; ++h) vh[h] = vhn[h];

        if (!(m.dbg & 1u)) dma_row(uniform(o2), enext2);
        mark(5);  // DMA issue
        if (m.dbg & 2u) asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
        else wait_keep_barrier((m.dbg & 1u) ? 0u : kdma);
    };

    float* const e0s = ering;
    float* const e1s = ering + erow;
    float* const e2s = ering + 2 * erow;
    while (true) {
        if (i >= len) break;
        step(e0s, e2s);
        if (++i >= len) break;
        step(e1s, e0s);
        if (++i >= len) break;
        step(e2s, e1s);
        ++i;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (STAMP) {
        if (lane == 0 && m.stamps) {
            mark(6);
            for (int k = 0; k < kBandStamps; ++k)
                m.stamps[((size_t)q * kMaxWaves + wave) * kBandStamps + k] = st_acc[k];
        }
    }

    // ---- epilogue: scores and the lowest-index argmin -------------------------------------
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
        for (uint32_t w = 1; w < W; ++w) lex_min(fv, fk, red[w], redk[w]);
        b.best[q] = (fk == 0xFFFFFFFFu) ? -1 : (int64_t)fk;
    }
}

template <int HA>
const void* band_ptr(int sm) {
    switch (sm) {
#define SVH_CASE(SMV) \
    case SMV: return reinterpret_cast<const void*>(&band_viterbi_kernel<SMV, HA>);
        SVH_CASE(1) SVH_CASE(2) SVH_CASE(3) SVH_CASE(4) SVH_CASE(5) SVH_CASE(6) SVH_CASE(8)
        SVH_CASE(10) SVH_CASE(12) SVH_CASE(16)
#undef SVH_CASE
        default: return nullptr;
    }
}

}  // namespace

hipError_t launch_band(const BandModel& m, int ha, const FusedBatch& b, hipStream_t stream) {
    const void* fn = ha == 1 ? band_ptr<1>((int)m.SM) : ha == 2 ? band_ptr<2>((int)m.SM) : nullptr;
    if ((m.dbg & 4u) && m.SM == 5 && ha == 1)
        fn = reinterpret_cast<const void*>(&band_viterbi_kernel<5, 1, true>);
    if (!fn) return hipErrorInvalidValue;
    if (b.nseq == 0) return hipSuccess;
    if (m.B == 0 || m.B % 64 || m.B > (uint32_t)kMaxBandThreads || m.erow % 256 ||
        m.erow < m.SM * m.B + kBandTail)
        return hipErrorInvalidValue;
    const size_t lds = band_lds_bytes(m.erow);
    if (lds > kMaxLdsBytes) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    BandModel mm = m;
    FusedBatch bb = b;
    void* args[] = {&mm, &bb};
    return hipLaunchKernel(fn, dim3(b.nseq), dim3(m.B), args, lds, stream);
}

}  // namespace svh
