// Device helpers shared by the HIP kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace svh {
namespace dev {

constexpr float kInf = __builtin_huge_valf();

// Workgroup barrier that only drains LDS/SMEM (lgkmcnt): in-flight global prefetches (the next
// emission row) stay in flight across it.  __syncthreads() would add vmcnt(0).  The "memory"
// clobber keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Wave-wide minimum, valid in lane 63.  Six DPP stages fused into v_min_f32_dpp (quad swaps,
// half-row / row mirrors, row broadcasts 15 and 31); rows masked off by row_mask keep their value,
// which is the identity for min.  s_nop 1 covers the VALU-write -> DPP-read hazard.
__device__ __forceinline__ float wave_min63(float x) {
    asm("s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(x));
    return x;
}

// Two independent chains interleaved (one wait state of distance between dependent DPP ops).
__device__ __forceinline__ void wave_min63x2(float& x, float& y) {
    asm("s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_min_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_min_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %1, %1, %1 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "v_min_f32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "v_min_f32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(x), "+v"(y));
}

// Lexicographic (value, index) minimum: lowest index among equal values (-0 == +0).
__device__ __forceinline__ void lex_min(float& v, uint32_t& k, float v2, uint32_t k2) {
    const bool take = (v2 < v) || (v2 == v && k2 < k);
    v = take ? v2 : v;
    k = take ? k2 : k;
}

template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ uint32_t dpp_u(uint32_t x, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, ROWMASK, 0xf, false);
}

template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ void lex_dpp_stage(float& v, uint32_t& k) {
    const float v2 = __builtin_bit_cast(float, dpp_u<CTRL, ROWMASK>(__builtin_bit_cast(uint32_t, v),
                                                                     0x7f800000u));
    const uint32_t k2 = dpp_u<CTRL, ROWMASK>(k, 0xFFFFFFFFu);
    lex_min(v, k, v2, k2);
}

// Lexicographic (value, index) wave minimum, valid in lane 63.
__device__ __forceinline__ void wave_lexmin63(float& v, uint32_t& k) {
    lex_dpp_stage<0xB1>(v, k);         // quad_perm [1,0,3,2]
    lex_dpp_stage<0x4E>(v, k);         // quad_perm [2,3,0,1]
    lex_dpp_stage<0x141>(v, k);        // row_half_mirror
    lex_dpp_stage<0x140>(v, k);        // row_mirror
    lex_dpp_stage<0x142, 0xa>(v, k);   // row_bcast:15
    lex_dpp_stage<0x143, 0xc>(v, k);   // row_bcast:31
}

// Order-preserving 64-bit key of (value, index): lexicographic (value, index) order becomes
// unsigned integer order, so one ds_min_u64 implements the argmin with lowest-index ties.
// -0 is folded into +0 (x + 0.0f) so that equal values compare equal.
__device__ __forceinline__ uint64_t lex_key(float v, uint32_t k) {
    uint32_t b = __builtin_bit_cast(uint32_t, v + 0.0f);
    b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    return ((uint64_t)b << 32) | k;
}
__device__ __forceinline__ float lex_key_value(uint64_t key) {
    uint32_t b = (uint32_t)(key >> 32);
    b = (b & 0x80000000u) ? (b & 0x7FFFFFFFu) : ~b;
    return __builtin_bit_cast(float, b);
}
__device__ __forceinline__ uint32_t lex_key_index(uint64_t key) { return (uint32_t)key; }

__device__ __forceinline__ void lds_atomic_min(float* p, float v) {
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_atomic_min(uint64_t* p, uint64_t v) {
    __hip_atomic_fetch_min(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ uint32_t align4(uint32_t x) { return (x + 3u) & ~3u; }

// LDS byte address of a pointer into dynamic LDS.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes land at
// lds_base + 16*l.  Issued from inline asm so the compiler does not treat every later LDS store
// as a possible alias of the in-flight DMA (it would insert vmcnt(0) before them); the caller
// retires it with a counted `s_waitcnt vmcnt` before the barrier that precedes the reads.
// M0 (reserved by the compiler) is saved and restored around the instruction.
__device__ __forceinline__ void lds_dma16(const void* gsrc, uint32_t lds_base_uniform) {
    uint32_t saved;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(saved)
        : "v"(gsrc), "s"(lds_base_uniform)
        : "memory");
}

// acc = (acc << 1) | bit per lane as v_addc_co_u32 acc, acc, acc with the compare's lane mask in
// VCC as the carry-in (hipcc's own code for the same C is four VALU ops: compare, shift, select,
// or).  push_le: bit = [x <= y]; push_lt_eqc: bit = [x < y] | (c & [x == y]), c a lane mask.
__device__ __forceinline__ void push_le(uint32_t& acc, float x, float y) {
    asm volatile("v_cmp_le_f32_e32 vcc, %1, %2\n\t"
                 "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
                 : "+v"(acc)
                 : "v"(x), "v"(y)
                 : "vcc");
}
__device__ __forceinline__ void push_lt_eqc(uint32_t& acc, float x, float y, uint64_t c) {
    uint64_t e;
    asm volatile("v_cmp_eq_f32_e64 %1, %2, %3\n\t"
                 "s_and_b64 %1, %1, %4\n\t"
                 "v_cmp_lt_f32_e32 vcc, %2, %3\n\t"
                 "s_or_b64 vcc, vcc, %1\n\t"
                 "v_addc_co_u32_e32 %0, vcc, %0, %0, vcc"
                 : "+v"(acc), "=&s"(e)
                 : "v"(x), "v"(y), "s"(c)
                 : "vcc", "scc");
}

}  // namespace dev
}  // namespace svh
