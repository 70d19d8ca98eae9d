// Instruction-cost microbenchmark for the pipelined kernel's step (gfx950, one wave per SIMD).
// Each test runs a block of 16 instructions `iters` times in one wave; the 4 waves of one
// 256-thread workgroup sit on the 4 SIMDs of one CU (the latency plan's occupancy).  Prints the
// shader cycles (s_memtime) per block, median over the waves.
//   hipcc --offload-arch=gfx950 -O3 -o build/isa_costs tools/ubench/isa_costs.hip && build/isa_costs
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

template <int T>
__global__ __launch_bounds__(256) void costs(float* out, unsigned long long* cyc, int iters, int nwaves) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float a = lane * 0.5f, b = 1.0f + lane, c = 2.0f, d = 3.0f, e = 4.0f, f = 5.0f, g = 6.0f, h = 7.0f;
    float tbl0 = lane, tbl1 = lane + 1, tbl2 = lane + 2, tbl3 = lane + 3;
    uint32_t acc = 0;
    const uint32_t idx = (uint32_t)__builtin_amdgcn_readfirstlane(lane + 3) & 15u;
    if (w >= nwaves) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if constexpr (T == 0) {  // 16 independent v_add_f32
            asm volatile(R4("v_add_f32 %0, %4, %5\n\tv_add_f32 %1, %4, %5\n\tv_add_f32 %2, %4, %5\n\tv_add_f32 %3, %4, %5\n\t")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
        } else if constexpr (T == 1) {  // 16 dependent v_add_f32
            asm volatile(R16("v_add_f32 %0, %0, %1\n\t") : "+v"(a) : "v"(b));
        } else if constexpr (T == 2) {  // 16 dependent v_min_f32
            asm volatile(R16("v_min_f32 %0, %0, %1\n\t") : "+v"(a) : "v"(b));
        } else if constexpr (T == 3) {  // 16 dependent v_pk_add_f32
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 p = {a, b}, q = {c, d};
            asm volatile(R16("v_pk_add_f32 %0, %0, %1\n\t") : "+v"(p) : "v"(q));
            a = p.x;
        } else if constexpr (T == 4) {  // 16 independent v_pk_add_f32
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 p = {a, b}, q = {c, d}, r = {e, f}, s = {g, h};
            asm volatile(R4("v_pk_add_f32 %0, %4, %4\n\tv_pk_add_f32 %1, %4, %4\n\tv_pk_add_f32 %2, %4, %4\n\tv_pk_add_f32 %3, %4, %4\n\t")
                         : "+v"(p), "+v"(q), "+v"(r), "+v"(s) : "v"(q));
            a = p.x + q.x + r.x + s.x;
        } else if constexpr (T == 5) {  // 8 x (v_readlane -> SGPR -> dependent v_add)
            uint32_t s;
            asm volatile(R4("v_readlane_b32 %1, %2, %3\n\tv_add_f32 %0, %1, %0\n\tv_readlane_b32 %1, %2, %3\n\tv_add_f32 %0, %1, %0\n\t")
                         : "+v"(a), "=&s"(s) : "v"(b), "s"(idx));
        } else if constexpr (T == 6) {  // 4 x (4 v_readlane, then 4 uses)
            uint32_t s0, s1, s2, s3;
            asm volatile(R4("v_readlane_b32 %1, %5, %9\n\tv_readlane_b32 %2, %6, %9\n\tv_readlane_b32 %3, %7, %9\n\tv_readlane_b32 %4, %8, %9\n\t"
                            "v_add_f32 %0, %1, %0\n\tv_add_f32 %0, %2, %0\n\tv_add_f32 %0, %3, %0\n\tv_add_f32 %0, %4, %0\n\t")
                         : "+v"(a), "=&s"(s0), "=&s"(s1), "=&s"(s2), "=&s"(s3)
                         : "v"(tbl0), "v"(tbl1), "v"(tbl2), "v"(tbl3), "s"(idx));
        } else if constexpr (T == 7) {  // 4 x (s_set_gpr_idx_on; 4 v_mov; s_set_gpr_idx_off) = 24 instructions
            asm volatile(R4("s_set_gpr_idx_on %4, gpr_idx(SRC0)\n\tv_mov_b32 %0, v0\n\tv_mov_b32 %1, v1\n\tv_mov_b32 %2, v2\n\tv_mov_b32 %3, v3\n\ts_set_gpr_idx_off\n\t")
                         : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : "s"(idx) : "m0");
        } else if constexpr (T == 8) {  // 8 x (v_cmp_lt vcc; v_addc vcc)
            asm volatile(R4("v_cmp_lt_f32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\tv_cmp_lt_f32 vcc, %2, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc\n\t")
                         : "+v"(acc) : "v"(a), "v"(b) : "vcc");
        } else if constexpr (T == 9) {  // 16 SALU
            uint32_t s = idx;
            asm volatile(R16("s_add_u32 %0, %0, 1\n\t") : "+s"(s) :: "scc");
            acc += s;
        } else if constexpr (T == 10) {  // 8 x (SALU; independent VALU)
            uint32_t s = idx;
            asm volatile(R4("s_add_u32 %0, %0, 1\n\tv_add_f32 %1, %3, %3\n\ts_add_u32 %0, %0, 1\n\tv_add_f32 %2, %3, %3\n\t")
                         : "+s"(s), "+v"(a), "+v"(b) : "v"(c) : "scc");
            acc += s;
        } else if constexpr (T == 11) {  // 8 x (v_add; dpp add reading the add 2 back: wave_shr), 2 chains
            asm volatile(R4("v_add_f32 %0, %2, %3\n\tv_add_f32 %1, %2, %3\n\tv_add_f32_dpp %2, %0, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n\tv_add_f32_dpp %3, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        } else if constexpr (T == 12) {  // 16 v_add_f32 with an SGPR operand written by SALU once per 4
            uint32_t s = idx;
            asm volatile(R4("s_add_u32 %1, %1, 1\n\tv_add_f32 %0, %1, %0\n\tv_add_f32 %0, %1, %0\n\tv_add_f32 %0, %1, %0\n\t")
                         : "+v"(a), "+s"(s) :: "scc");
        } else if constexpr (T == 13) {  // 16 independent v_mov_b32
            asm volatile(R4("v_mov_b32 %0, %4\n\tv_mov_b32 %1, %4\n\tv_mov_b32 %2, %4\n\tv_mov_b32 %3, %4\n\t")
                         : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : "v"(e));
        } else if constexpr (T == 14) {  // 8 x (ds_write_b32 + v_add) independent
            const uint32_t ad = lane * 4;
            asm volatile(R4("ds_write_b32 %2, %1\n\tv_add_f32 %0, %1, %0\n\tds_write_b32 %2, %1 offset:256\n\tv_add_f32 %0, %1, %0\n\t")
                         : "+v"(a) : "v"(b), "v"(ad) : "memory");
        } else if constexpr (T == 15) {  // 16 independent v_min_f32
            asm volatile(R4("v_min_f32 %0, %4, %5\n\tv_min_f32 %1, %4, %5\n\tv_min_f32 %2, %4, %5\n\tv_min_f32 %3, %4, %5\n\t")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
        } else if constexpr (T == 16) {  // 8 x dependent pair (v_add; v_min) = the chain recurrence
            asm volatile(R4("v_add_f32 %0, %1, %0\n\tv_min_f32 %0, %2, %0\n\tv_add_f32 %0, %1, %0\n\tv_min_f32 %0, %2, %0\n\t")
                         : "+v"(a) : "v"(b), "v"(c));
        } else if constexpr (T == 17) {  // 16 v_add_f32 reading an SGPR written by v_readlane 4+ instructions earlier
            uint32_t s0, s1;
            asm volatile(R4("v_readlane_b32 %1, %3, %4\n\tv_add_f32 %0, %2, %0\n\tv_add_f32 %0, %2, %0\n\tv_add_f32 %0, %2, %0\n\t"
                            "v_readlane_b32 %2, %3, %4\n\tv_add_f32 %0, %1, %0\n\tv_add_f32 %0, %1, %0\n\tv_add_f32 %0, %1, %0\n\t")
                         : "+v"(a), "=&s"(s0), "=&s"(s1) : "v"(b), "s"(idx));
        } else if constexpr (T == 18) {  // 16 independent v_add_f32 with s_nop 0 after each 4 (issue cost of s_nop)
            asm volatile(R4("v_add_f32 %0, %4, %5\n\tv_add_f32 %1, %4, %5\n\tv_add_f32 %2, %4, %5\n\ts_nop 0\n\t")
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e), "v"(f));
        } else if constexpr (T == 19) {  // 4 x (s_set_gpr_idx_on SRC0; 4 v_mov; off) then an immediate dependent use
            asm volatile(R4("s_set_gpr_idx_on %5, gpr_idx(SRC0)\n\tv_mov_b32 %0, v0\n\tv_mov_b32 %1, v1\n\tv_mov_b32 %2, v2\n\tv_mov_b32 %3, v3\n\ts_set_gpr_idx_off\n\tv_add_f32 %4, %0, %4\n\t")
                         : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d), "+v"(e) : "s"(idx) : "m0");
        } else if constexpr (T == 20) {  // s_movrels_b32 from an SGPR table (M0-indexed SALU move), 16 x
            uint32_t s;
            asm volatile("s_mov_b32 m0, %1\n\t" R16("s_movrels_b32 %0, s0\n\t") : "=&s"(s) : "s"(idx) : "m0");
            acc += s;
        } else if constexpr (T == 21) {  // 16 independent v_add_f32_dpp row_ror (sources not recently written)
            asm volatile(R4("v_add_f32_dpp %0, %4, %5 row_ror:3 row_mask:0xf bank_mask:0xf\n\tv_add_f32_dpp %1, %4, %5 row_ror:3 row_mask:0xf bank_mask:0xf\n\tv_add_f32_dpp %2, %4, %5 row_ror:3 row_mask:0xf bank_mask:0xf\n\tv_add_f32_dpp %3, %4, %5 row_ror:3 row_mask:0xf bank_mask:0xf\n\t")
                         : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d) : "v"(e), "v"(f));
        } else if constexpr (T == 22) {  // ds_read_b128 broadcast then wait: latency round trip x 4
            const uint32_t ad = 0;
            typedef float f4 __attribute__((ext_vector_type(4)));
            f4 r;
            asm volatile(R4("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)\n\t") : "=&v"(r) : "v"(ad) : "memory");
            a = r.x;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = a + b + c + d + e + f + g + h + tbl0 + tbl1 + tbl2 + tbl3 + (float)acc;
}

template <int T>
double run(int iters, int nwaves, float* dout, unsigned long long* dcyc) {
    hipLaunchKernelGGL(costs<T>, dim3(1), dim3(256), 0, 0, dout, dcyc, iters, nwaves);
    hipLaunchKernelGGL(costs<T>, dim3(1), dim3(256), 0, 0, dout, dcyc, iters, nwaves);
    std::vector<unsigned long long> h(4);
    hipMemcpy(h.data(), dcyc, 32, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.begin() + nwaves);
    return (double)h[nwaves / 2] / iters;
}

int main() {
    float* dout;
    unsigned long long* dcyc;
    hipMalloc(&dout, 256 * 4);
    hipMalloc(&dcyc, 64);
    hipMemset(dcyc, 0, 64);
    const int it = 4096;
    const char* names[] = {"16 indep v_add_f32", "16 dep v_add_f32", "16 dep v_min_f32", "16 dep v_pk_add_f32",
                           "16 indep v_pk_add_f32", "8x(v_readlane->dep v_add)", "4x(4 readlane,4 uses)",
                           "4x(idx_on,4 v_mov,idx_off)", "8x(v_cmp vcc, v_addc)", "16 SALU dep", "8x(SALU,VALU)",
                           "8x(add,dpp add) 2 chains", "4x(SALU write s, 3 v_add read s)", "16 indep v_mov",
                           "8x(ds_write_b32, v_add)", "16 indep v_min_f32", "8x(dep v_add, v_min)",
                           "16 v_add + 2 readlane (4 apart)", "12 v_add + 4 s_nop0", "4x(idx block + dep use)",
                           "16 s_movrels", "16 indep dpp row_ror adds", "4x(ds_read_b128 + lgkmcnt0)"};
    double r[2][23];
    for (int nw = 1; nw <= 4; nw += 3) {
        const int k = nw == 1 ? 0 : 1;
        r[k][0] = run<0>(it, nw, dout, dcyc);
        r[k][1] = run<1>(it, nw, dout, dcyc);
        r[k][2] = run<2>(it, nw, dout, dcyc);
        r[k][3] = run<3>(it, nw, dout, dcyc);
        r[k][4] = run<4>(it, nw, dout, dcyc);
        r[k][5] = run<5>(it, nw, dout, dcyc);
        r[k][6] = run<6>(it, nw, dout, dcyc);
        r[k][7] = run<7>(it, nw, dout, dcyc);
        r[k][8] = run<8>(it, nw, dout, dcyc);
        r[k][9] = run<9>(it, nw, dout, dcyc);
        r[k][10] = run<10>(it, nw, dout, dcyc);
        r[k][11] = run<11>(it, nw, dout, dcyc);
        r[k][12] = run<12>(it, nw, dout, dcyc);
        r[k][13] = run<13>(it, nw, dout, dcyc);
        r[k][14] = run<14>(it, nw, dout, dcyc);
        r[k][15] = run<15>(it, nw, dout, dcyc);
        r[k][16] = run<16>(it, nw, dout, dcyc);
        r[k][17] = run<17>(it, nw, dout, dcyc);
        r[k][18] = run<18>(it, nw, dout, dcyc);
        r[k][19] = run<19>(it, nw, dout, dcyc);
        r[k][20] = run<20>(it, nw, dout, dcyc);
        r[k][21] = run<21>(it, nw, dout, dcyc);
        r[k][22] = run<22>(it, nw, dout, dcyc);
    }
    const hipError_t e = hipDeviceSynchronize();
    std::printf("status %s\n%-36s %10s %10s\n", hipGetErrorString(e), "block", "1 wave", "4 waves");
    for (int i = 0; i < 23; ++i) std::printf("%-36s %10.1f %10.1f\n", names[i], r[0][i], r[1][i]);
    return 0;
}
