// Device helpers shared by the pipelined chain kernels (pipe.hip: latency plan, pipe_wide.hip:
// throughput plan).  Boundary granules are 8-byte {score, tag} words in an L2 ring per sequence
// boundary; agent-scope relaxed accesses (sc1) keep them coherent across CUs.
#pragma once
#include "device_common.h"
#include "kernels.h"

namespace svh {
namespace pipe_dev {

constexpr uint32_t kGR = kPipeGRing;
constexpr uint32_t kSpinLimit = 1u << 22;
constexpr uint32_t kNoRow = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t lds_ld32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Agent-scope relaxed accesses: global_load / global_store ... sc1 (L2-coherent, bypass L1).
__device__ __forceinline__ uint64_t g_ld64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_st64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A score that a re-run on another XCD may overwrite in the same launch (the in-kernel re-run of a
// row whose speculation failed): an agent-scope store, written through to memory, not left dirty in
// this XCD's L2 -- the L2s are not coherent, and a dirty line written back after the re-run's stores
// would put the speculated value back (measured: rows re-run from another XCD came out wrong
// intermittently on the diagonal plan, tools/diag_stress.py).
__device__ __forceinline__ void g_st_score(float* p, float v) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float readlane_f(float x, uint32_t l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), (int)l));
}
__device__ __forceinline__ uint32_t readlane_u(uint32_t x, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}

// Granule tag of observation s in this launch: epoch and ring lap (a slot is rewritten every
// kGR observations; flow control keeps the consumer within one lap).
__device__ __forceinline__ uint32_t gtag(uint32_t ep, uint32_t s) {
    return ((ep % 0xFFFFFu + 1u) << 12) | ((s >> 8) & 0xFFFu);  // never 0 (zeroed memory)
}
static_assert(kGR == 256, "gtag assumes a 256-slot ring");

// Granule prefetch into a register the loop carries (tied operand: no copy at the back edge, so
// no wait is forced there); the caller waits with an explicit vmcnt before reading it.
__device__ __forceinline__ void g_prefetch64(uint64_t& dst, const uint64_t* p) {
    asm volatile("global_load_dwordx2 %0, %1, off sc1" : "+v"(dst) : "v"(p) : "memory");
}

// The last workgroup of a launch to finish (every one has taken its ticket and read the epoch):
// tickets and the finish count back to 0, the epoch advanced (ctr[2] + 1 is this launch's).
__device__ __forceinline__ void pipe_reset_counters(const PipeScratch& x) {
    const uint32_t ep = __hip_atomic_load(x.ctr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __hip_atomic_store(x.ctr + 0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(x.ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t c = kCtrClass; c <= kCtrLeft; ++c) __hip_atomic_store(x.ctr + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(x.ctr + 2, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// hwreg(HW_REG_XCC_ID, 0, 4): the XCD this wave runs on (the XCD-local hand-offs, SVH_PIPE_XL)
__device__ __forceinline__ uint32_t xcc_id() { return (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xFu; }

}  // namespace pipe_dev
}  // namespace svh
