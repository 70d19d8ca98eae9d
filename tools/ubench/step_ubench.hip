// Step-level microbenchmark of the pipelined latency kernel (pipe.hip, SM = 2): one wave per SIMD,
// 4 waves per workgroup, no exchange (the boundary input is a constant vector), tables in VGPRs.
// Each variant runs `groups` x 32 observations; prints shader cycles per observation (median over
// waves and workgroups) and checks that every variant's final state equals variant 0's.
//   hipcc --offload-arch=gfx950 -O3 -fno-honor-nans -o tools/ubench/step_ubench tools/ubench/step_ubench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef float f32x32 __attribute__((ext_vector_type(32)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float readlane_f(float x, uint32_t l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), (int)l));
}
__device__ __forceinline__ uint32_t readlane_u(uint32_t x, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}

template <int R>
__device__ __forceinline__ void chain_terms_v(float& xb, float& xa, float eb, float ea, float bvv, float f, float x) {
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
            : "v"(bvv), "v"(eb), "v"(f), "v"(ea), "v"(x), "n"(16 - R));
    }
}
// xb only (the chain term of slot 0), for variants that form xa by a packed add
template <int R>
__device__ __forceinline__ float chain_b(float eb, float bvv, float x) {
    float xb;
    if constexpr (R == 0) {
        asm("v_add_f32_e32 %0, %1, %2\n\t"
            "v_add_f32_dpp %0, %3, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb)
            : "v"(bvv), "v"(eb), "v"(x));
    } else {
        asm("v_add_f32_dpp %0, %1, %2 row_ror:%4 row_mask:0xf bank_mask:0xf\n\t"
            "v_add_f32_dpp %0, %3, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "=&v"(xb)
            : "v"(bvv), "v"(eb), "v"(x), "n"(16 - R));
    }
    return xb;
}

// Pair tables (S <= 20, M0 = 2o): table k at v[2 + 40k ..], register 2o + u = value u of symbol o.
//   V1..V3: P0 = {eb0, ea0}, P1 = {eb1, ea1}, P2 = {A_S, A_F}, P3 = {X_SS, X_FF}
//   V5:     P0 = {ea0, ea1}, P1 = {eb0, eb1}, P2, P3 as above
#define TAB_IN "{v[2:33]}"(TA[0]), "{v[34:41]}"(TB[0]), "{v[42:73]}"(TA[1]), "{v[74:81]}"(TB[1]), \
               "{v[82:113]}"(TA[2]), "{v[114:121]}"(TB[2]), "{v[122:153]}"(TA[3]), "{v[154:161]}"(TB[3])

struct St {
    float v0, v1, cx, cy, extra;
};

template <int V>
__global__ __launch_bounds__(256) void steps(const float* tab, const uint8_t* syms, float* out,
                                             unsigned long long* cyc, int groups, int S) {
    extern __shared__ float lds[];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * 4 + w;
    // tables: per (slot, symbol) the lane's eb, ea; per symbol the heavy constants
    // tab layout: [slot][o][64] eb, then ea, then consts [o][4]
    const float* teb[2] = {tab + 0 * 32 * 64, tab + 1 * 32 * 64};
    const float* tea[2] = {tab + 2 * 32 * 64, tab + 3 * 32 * 64};
    const float* hc = tab + 4 * 32 * 64;
    f32x32 EB[2], EA[2];
    f32x32 TA[4];
    f32x8 TB[4];
    constexpr bool pair = V >= 1;
    if constexpr (!pair) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int o = 0; o < 32; ++o) {
                EB[s][o] = teb[s][o * 64 + lane];
                EA[s][o] = tea[s][o * 64 + lane];
            }
    } else {
#pragma unroll
        for (int o = 0; o < 20; ++o) {
            float val[4][2];
            if constexpr (V == 5) {
                val[0][0] = tea[0][o * 64 + lane], val[0][1] = tea[1][o * 64 + lane];
                val[1][0] = teb[0][o * 64 + lane], val[1][1] = teb[1][o * 64 + lane];
            } else {
                val[0][0] = teb[0][o * 64 + lane], val[0][1] = tea[0][o * 64 + lane];
                val[1][0] = teb[1][o * 64 + lane], val[1][1] = tea[1][o * 64 + lane];
            }
            val[2][0] = hc[o * 4 + 0], val[2][1] = hc[o * 4 + 1];
            val[3][0] = hc[o * 4 + 2], val[3][1] = hc[o * 4 + 3];
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int r = 2 * o + u;
                    if (r < 32) TA[k][r] = val[k][u];
                    else TB[k][r - 32] = val[k][u];
                }
        }
        // opaque per-lane values (the heavy constants are uniform: the compiler would keep them
        // in SGPRs and copy them into the pinned registers at every step)
#pragma unroll
        for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(TA[k]), "+v"(TB[k]));
    }
    const bool lo = lane < (uint32_t)S;
    const float cAS = lo ? hc[lane * 4 + 0] : INFINITY, cAF = lo ? hc[lane * 4 + 1] : INFINITY;
    const float cXSS = lo ? hc[lane * 4 + 2] : INFINITY, cXFF = lo ? hc[lane * 4 + 3] : INFINITY;

    float v[2] = {tab[lane] * 0.5f, tab[64 + lane] * 0.5f};
    f2 CF = {lane == 0 ? 1.0f : INFINITY, 0.25f};
    uint32_t viol = 0;
    float vmin = INFINITY;  // V2+: min of fl(A_F + m) - F'
    const float bconst = 3.0f + (float)lane;  // the boundary vector (no exchange)
    float* ring = lds + w * 32 * 64;
    float bv_prev = bconst;

    auto step = [&](uint32_t o, auto rc, float bv) {
        constexpr int R = decltype(rc)::value;
        float xa[2], xb[2];
        f2 kS, kX;  // {A_S, A_F}, {X_SS, X_FF}
        if constexpr (V == 0) {
            kS = (f2){readlane_f(cAS, o), readlane_f(cAF, o)};
            kX = (f2){readlane_f(cXSS, o), readlane_f(cXFF, o)};
            float eb[2], ea[2];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                eb[s] = EB[s][o];
                ea[s] = EA[s][o];
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) asm volatile("" : "+v"(eb[s]), "+v"(ea[s]));
            chain_terms_v<R>(xb[0], xa[0], eb[0], ea[0], bv, CF.y, v[1]);
            xa[1] = ea[1] + CF.y;
            xb[1] = eb[1] + v[0];
        } else if constexpr (V == 7) {  // indexed operands in one SRC0 block (pair tables)
            const float pm0 = fminf(v[0], v[1]);
            f2 pmv;  // the packed add reads the low half twice (op_sel_hi): the high half stays undefined
            pmv.x = pm0;
            float eb0;
            f2 s1v, s2v;
            asm volatile("s_set_gpr_idx_on %[o], gpr_idx(SRC0)\n\t"
                         "v_mov_b32 %[eb0], v2\n\t"
                         "v_add_f32 %[xa0], v3, %[f]\n\t"
                         "v_add_f32 %[xa1], v43, %[f]\n\t"
                         "v_add_f32 %[xb1], v42, %[v0]\n\t"
                         "v_pk_add_f32 %[s1], v[82:83], %[pm] op_sel_hi:[1,0]\n\t"
                         "v_pk_add_f32 %[s2], v[122:123], %[cf]\n\t"
                         "s_set_gpr_idx_off"
                         : [eb0] "=&v"(eb0), [xa0] "=&v"(xa[0]), [xa1] "=&v"(xa[1]), [xb1] "=&v"(xb[1]),
                           [s1] "=&v"(s1v), [s2] "=&v"(s2v)
                         : [o] "s"(2 * o), [f] "v"(CF.y), [v0] "v"(v[0]), [pm] "v"(pmv), [cf] "v"(CF), TAB_IN
                         : "m0");
            xb[0] = chain_b<R>(eb0, bv, v[1]);
            const float n0 = fminf(xa[0], xb[0]), n1 = fminf(xa[1], xb[1]);
            const float cn = fminf(s1v.x, s2v.x);
            asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, 0, %0, vcc"
                         : "+v"(viol)
                         : "v"(s1v.y), "v"(s2v.y)
                         : "vcc");
            CF = (f2){cn, s2v.y};
            v[0] = n0;
            v[1] = n1;
            return;
        } else {
            f2 p0, p1;
            if constexpr (V == 4) {  // eight 32-bit moves
                float e0, a0, e1, a1, s0, s1, x0, x1;
                asm volatile("s_set_gpr_idx_on %[o], gpr_idx(SRC0)\n\t"
                             "v_mov_b32 %[e0], v2\n\tv_mov_b32 %[a0], v3\n\t"
                             "v_mov_b32 %[e1], v42\n\tv_mov_b32 %[a1], v43\n\t"
                             "v_mov_b32 %[s0], v82\n\tv_mov_b32 %[s1], v83\n\t"
                             "v_mov_b32 %[x0], v122\n\tv_mov_b32 %[x1], v123\n\t"
                             "s_set_gpr_idx_off"
                             : [e0] "=&v"(e0), [a0] "=&v"(a0), [e1] "=&v"(e1), [a1] "=&v"(a1), [s0] "=&v"(s0),
                               [s1] "=&v"(s1), [x0] "=&v"(x0), [x1] "=&v"(x1)
                             : [o] "s"(2 * o), TAB_IN
                             : "m0");
                p0 = (f2){e0, a0};
                p1 = (f2){e1, a1};
                kS = (f2){s0, s1};
                kX = (f2){x0, x1};
            } else {  // four 64-bit moves
                asm volatile("s_set_gpr_idx_on %[o], gpr_idx(SRC0)\n\t"
                             "v_mov_b64 %[p0], v[2:3]\n\tv_mov_b64 %[p1], v[42:43]\n\t"
                             "v_mov_b64 %[ks], v[82:83]\n\tv_mov_b64 %[kx], v[122:123]\n\t"
                             "s_set_gpr_idx_off"
                             : [p0] "=&v"(p0), [p1] "=&v"(p1), [ks] "=&v"(kS), [kx] "=&v"(kX)
                             : [o] "s"(2 * o), TAB_IN
                             : "m0");
            }
            if constexpr (V == 5) {  // p0 = {ea0, ea1}, p1 = {eb0, eb1}
                const f2 xa2 = p0 + (f2){CF.y, CF.y};
                xa[0] = xa2.x;
                xa[1] = xa2.y;
                xb[0] = chain_b<R>(p1.x, bv, v[1]);
                xb[1] = p1.y + v[0];
            } else {
                chain_terms_v<R>(xb[0], xa[0], p0.x, p0.y, bv, CF.y, v[1]);
                xa[1] = p1.y + CF.y;
                xb[1] = p1.x + v[0];
            }
        }
        const float n0 = fminf(xa[0], xb[0]), n1 = fminf(xa[1], xb[1]);
        const float pm = fminf(v[0], v[1]);
        const f2 s1 = kS + (f2){pm, pm};
        const f2 s2 = kX + CF;
        const float cn = fminf(s1.x, s2.x);
        if constexpr (V <= 1 || V >= 6) {
            asm volatile("v_cmp_lt_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, 0, %0, vcc"
                         : "+v"(viol)
                         : "v"(s1.y), "v"(s2.y)
                         : "vcc");
        } else {
            float d;
            asm volatile("v_sub_f32_e32 %1, %2, %3\n\tv_min_f32_e32 %0, %0, %1" : "+v"(vmin), "=&v"(d) : "v"(s1.y), "v"(s2.y));
        }
        CF = (f2){cn, s2.y};
        v[0] = n0;
        v[1] = n1;
    };

    uint4 cw = *reinterpret_cast<const uint4*>(syms + lane * 16);
    asm volatile("" ::"v"(cw.x), "v"(cw.y), "v"(cw.z), "v"(cw.w));
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < groups; ++it) {
        const uint32_t ln = (uint32_t)(2 * (it & 31));
        const uint64_t sw[4] = {(uint64_t)readlane_u(cw.x, ln) | ((uint64_t)readlane_u(cw.y, ln) << 32),
                                (uint64_t)readlane_u(cw.z, ln) | ((uint64_t)readlane_u(cw.w, ln) << 32),
                                (uint64_t)readlane_u(cw.x, ln + 1) | ((uint64_t)readlane_u(cw.y, ln + 1) << 32),
                                (uint64_t)readlane_u(cw.z, ln + 1) | ((uint64_t)readlane_u(cw.w, ln + 1) << 32)};
        auto group = [&](auto jc) {
            constexpr uint32_t j = decltype(jc)::value;
            const float bv = bconst + (float)j;
            auto one = [&](auto kc) {
                constexpr uint32_t k = decltype(kc)::value;
                const uint32_t o = (uint32_t)((sw[j] >> (8 * k)) & 0xFFu);
                if constexpr (k == 0) step(o, std::integral_constant<int, 7>{}, bv_prev);
                else step(o, std::integral_constant<int, (int)k - 1>{}, bv);
                if constexpr (V != 3 && V != 6 && V != 8) ring[(8 * j + k) * 64 + lane] = v[1];
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
        };
        group(std::integral_constant<uint32_t, 0>{});
        group(std::integral_constant<uint32_t, 1>{});
        group(std::integral_constant<uint32_t, 2>{});
        group(std::integral_constant<uint32_t, 3>{});
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[gw] = t1 - t0;
    const bool bad = V <= 1 || V >= 6 ? viol != 0 : vmin < 0.0f;
    St* o = reinterpret_cast<St*>(out) + gw * 64 + lane;
    o->v0 = v[0];
    o->v1 = v[1];
    o->cx = CF.x;
    o->cy = CF.y;
    o->extra = bad ? 1.0f : 0.0f;
}

template <int V>
double run(const float* dtab, const uint8_t* dsym, float* dout, unsigned long long* dcyc, int groups, int blocks,
           std::vector<St>& res) {
    const size_t lds = 4 * 32 * 64 * 4;
    for (int r = 0; r < 2; ++r)
        hipLaunchKernelGGL(steps<V>, dim3(blocks), dim3(256), lds, 0, dtab, dsym, dout, dcyc, groups, 20);
    std::vector<unsigned long long> h(blocks * 4);
    hipMemcpy(h.data(), dcyc, h.size() * 8, hipMemcpyDeviceToHost);
    res.resize(blocks * 4 * 64);
    hipMemcpy(res.data(), dout, res.size() * sizeof(St), hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    return (double)h[h.size() / 2] / (groups * 32.0);
}

int main(int argc, char** argv) {
    const int groups = 2048, blocks = argc > 1 ? atoi(argv[1]) : 1;
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> ud(0.5f, 6.0f);
    std::vector<float> tab(4 * 32 * 64 + 32 * 4);
    for (auto& x : tab) x = ud(rng);
    for (int o = 20; o < 32; ++o)
        for (int s = 0; s < 4; ++s)
            for (int l = 0; l < 64; ++l) tab[(s * 32 + o) * 64 + l] = INFINITY;
    // heavy constants: A_S, A_F large (the light term rarely wins), X_SS, X_FF small
    for (int o = 0; o < 32; ++o) {
        tab[4 * 32 * 64 + o * 4 + 0] = o < 20 ? 9.0f + ud(rng) : INFINITY;
        tab[4 * 32 * 64 + o * 4 + 1] = o < 20 ? 11.0f + ud(rng) : INFINITY;
        tab[4 * 32 * 64 + o * 4 + 2] = o < 20 ? 0.01f * ud(rng) : INFINITY;
        tab[4 * 32 * 64 + o * 4 + 3] = o < 20 ? 0.01f * ud(rng) : INFINITY;
    }
    std::vector<uint8_t> sym(1024);
    for (auto& s : sym) s = rng() % 20;
    float *dtab, *dout;
    uint8_t* dsym;
    unsigned long long* dcyc;
    hipMalloc(&dtab, tab.size() * 4);
    hipMalloc(&dsym, sym.size());
    hipMalloc(&dout, (size_t)blocks * 256 * sizeof(St));
    hipMalloc(&dcyc, (size_t)blocks * 4 * 8);
    hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dsym, sym.data(), sym.size(), hipMemcpyHostToDevice);
    const char* names[] = {"V0 current (readlane consts, cmp/addc, ds_write)",
                           "V1 4x v_mov_b64 pair tables, cmp/addc, ds_write",
                           "V2 V1 + sub/min check",
                           "V3 V2 without ds_write",
                           "V4 8x v_mov_b32 pair tables, sub/min, ds_write",
                           "V5 V2 + packed xa pair",
                           "V6 V0 without ds_write",
                           "V7 indexed operands in one SRC0 block, ds_write"};
    std::vector<St> ref, got;
    double c[8];
    c[0] = run<0>(dtab, dsym, dout, dcyc, groups, blocks, ref);
    bool same[8] = {true};
    auto cmp = [&](int i) {
        same[i] = true;
        for (size_t k = 0; k < ref.size(); ++k)
            if (std::memcmp(&ref[k], &got[k], sizeof(St)) != 0) {
                same[i] = false;
                break;
            }
    };
    c[1] = run<1>(dtab, dsym, dout, dcyc, groups, blocks, got), cmp(1);
    c[2] = run<2>(dtab, dsym, dout, dcyc, groups, blocks, got), cmp(2);
    c[3] = run<3>(dtab, dsym, dout, dcyc, groups, blocks, got), cmp(3);
    c[4] = run<4>(dtab, dsym, dout, dcyc, groups, blocks, got), cmp(4);
    c[5] = run<5>(dtab, dsym, dout, dcyc, groups, blocks, got), cmp(5);
    c[6] = run<6>(dtab, dsym, dout, dcyc, groups, blocks, got), cmp(6);
    c[7] = run<7>(dtab, dsym, dout, dcyc, groups, blocks, got), cmp(7);
    const hipError_t e = hipDeviceSynchronize();
    std::printf("status %s, %d workgroup(s) of 4 waves, %d observations\n", hipGetErrorString(e), blocks, groups * 32);
    for (int i = 0; i < 8; ++i)
        std::printf("%-52s %7.1f cycles/obs  %s\n", names[i], c[i], same[i] ? "same state" : "DIFFERS");
    std::printf("ref lane0: v0 %g v1 %g c %g F %g viol %g\n", ref[0].v0, ref[0].v1, ref[0].cx, ref[0].cy, ref[0].extra);
    return 0;
}
