// Host runtime of the engine: HMM -> device model (plan + HBM upload), batches, _spec products.
// Used by the C ABI (svh_api.cpp).  Errors are reported by throwing svh::Error.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "error.h"
#include "kernels.h"
#include "svh.h"

namespace svh {


void hip_check(hipError_t e, const char* what);

// Restores the caller's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev);
    ~DeviceGuard();
};

// Device allocation owned by RAII.
struct DeviceBuffer {
    void* ptr = nullptr;
    size_t bytes = 0;
    DeviceBuffer() = default;
    DeviceBuffer(const DeviceBuffer&) = delete;
    DeviceBuffer& operator=(const DeviceBuffer&) = delete;
    DeviceBuffer(DeviceBuffer&& o) noexcept : ptr(o.ptr), bytes(o.bytes) { o.ptr = nullptr; o.bytes = 0; }
    DeviceBuffer& operator=(DeviceBuffer&& o) noexcept;
    ~DeviceBuffer();
    void alloc(size_t nbytes);
    void upload(const void* src, size_t nbytes, hipStream_t s);
    void reserve(size_t nbytes);  // grow-only (keeps the allocation when large enough)
    void upload_async(const void* src, size_t nbytes, hipStream_t s);  // reserve + async copy
    template <class T> T* as() const { return static_cast<T*>(ptr); }
};

// Canonical host form of the model (reference semantics resolved: dense start with first
// duplicate winning, CSR of T^T with first duplicate winning, columns ascending).
struct HostModel {
    uint32_t n = 0, S = 0;
    std::vector<float> start;     // n
    std::vector<float> emis;      // S * n
    std::vector<uint32_t> rowptr; // n + 1
    std::vector<uint32_t> col;    // nnz
    std::vector<float> val;       // nnz
    uint32_t nnz() const { return (uint32_t)col.size(); }
};

HostModel build_host_model(uint64_t n, uint64_t S, uint64_t nstart, const uint64_t* start_cols,
                           const float* start_vals, const float* emissions, uint64_t ntrans,
                           const uint64_t* src, const uint64_t* dst, const float* prob);

// Register/LDS schedule of the fused kernel.
struct Plan {
    bool fused = false;
    int family = -1;
    uint32_t B = 0, SM = 0, R = 0, HM = 0, XM = 0, H = 0;
    int mode = kHeavyGeneral;
    uint32_t estride = 0, vstride = 0;
    int hrow[kMaxHeavy] = {0, 0, 0, 0};
    float hw[kMaxHeavy] = {0, 0, 0, 0};
    uint32_t xk[kMaxHeavy][kMaxExc] = {};
    float xw[kMaxHeavy][kMaxExc] = {};
    std::vector<uint32_t> lcol;
    std::vector<float> lval;
    std::vector<float> hval;
    std::vector<uint8_t> hvalid;
    std::vector<float> hmask;
    std::vector<float> emis_pad;   // S * estride (+ tail)
    std::vector<float> start_pad;  // estride + 16
    size_t lds_bytes = 0;
};

// Build the fused plan, or return plan.fused == false when no family fits.  allow_uniform=false
// restricts to term-by-term heavy rows (needed for argmin backpointers).
Plan make_plan(const HostModel& hm, int max_threads, bool allow_uniform);

// A plan resident in HBM plus the kernel-argument view of it.
struct DevicePlan {
    Plan plan;
    DeviceBuffer d_emis, d_start, d_lcol, d_lval, d_hval, d_hvalid, d_hmask;
    FusedModel view{};
    void upload(const Plan& p, hipStream_t s);
};

// Host schedule of the chain ("band") kernel (band.hip); ok == false when the model does not
// have the chain + uniform-heavy shape.
struct BandPlan {
    bool ok = false;
    bool chain = false;  // barrier-free register kernel (chain.hip) instead of band.hip
    bool ge = false;     // chain kernel streams E rows from L2 (erows_t) instead of VGPRs
    uint32_t B = 0, SM = 0, HA = 0, H = 0, nL = 0, erow = 0;
    int hrow[kBandHeavy] = {0, 0};
    int hvalid[kBandHeavy] = {0, 0};
    float hstart[kBandHeavy] = {0, 0};
    std::vector<float> erows, erows_t, start, aw, bw;
    std::vector<uint32_t> lrow;
    std::vector<uint8_t> pflags;  // decoded paths (BandModel::pflags)
    std::vector<int32_t> spos;    // decoded paths (BandModel::spos)
    uint32_t hx_exist = 0, hl_exist = 0;
    bool ties_heavy = false;  // every light position has a heavy term that wins ties (BandModel)
    size_t lds_bytes = 0;
    // the decoded-path chain variant can run this plan
    bool paths_ok() const { return ok && chain && !ge && HA <= 1 && chain_paths_supported((int)SM, (int)(B / 64)); }
};
// ge_waves: -1 = SVH_CHAIN_GE (diagnostic) or none; 0 = none; w > 0 = streamed-E chain kernel
// with w waves.
BandPlan make_band_plan(const HostModel& hm, int max_threads, bool chain, int ge_waves = -1);

struct DeviceBandPlan {
    BandPlan plan;
    DeviceBuffer d_erows, d_erows_t, d_start, d_aw, d_bw, d_lrow, d_stamps, d_pflags, d_spos;
    BandModel view{};
    void upload(const BandPlan& p, uint32_t n, uint32_t S, hipStream_t s);
    void report_stamps(uint32_t nseq) const;  // diagnostic (SVH_BAND_DEBUG & 4)
};

// Host tables of the pipelined chain kernel (pipe.hip); ok == false when the model does not
// qualify (kernels.h, PipeModel).
struct PipePlan {
    bool ok = false;
    bool sx = false;
    uint32_t SM = 0, W = 0, G = 0, nblk = 0, P = 0;
    int rowF = -1, rowS = -1;
    float startF = 0, startS = 0;
    std::vector<float> tab;     // [nblk][S][SM][64][2]
    std::vector<float> e0;      // [S][P]
    std::vector<float> start;   // [P]
    std::vector<uint32_t> lrow; // [P]
    std::vector<float> hc;      // [S][8]
    bool wide = false;          // pipe_wide.hip layout: tab [nblk][S][SM/2][64][4], W sequences per workgroup
    // diagonal plan (diag.hip; latency plan only): [S][64 nrng] float2 {ea, eb}, +inf past the light rows
    std::vector<float> dtab;
    uint32_t nrng = 0;
    // _spec level 2 on this plan (pipe_l2.hip): the largest finite ea = fl(E_o[p] + aw_p), or +inf
    // when some score is negative (its margin check needs every score >= 0) or the plan is wide
    float emax2 = 0.0f;
    // decoded paths (PipeModel::pflags / spos / hx_exist / hl_exist / ties_heavy)
    std::vector<uint8_t> pflags;  // [P]
    std::vector<int32_t> spos;    // [n]
    uint32_t hx_exist = 0, hl_exist = 0;
    bool ties_heavy = false;
};
// sm = 0 / waves = 0: defaults (SVH_PIPE_SM / SVH_PIPE_WAVES override them, diagnostics)
PipePlan make_pipe_plan(const HostModel& hm, uint32_t sm = 0, uint32_t waves = 0, bool wide = false);

struct DevicePipePlan {
    PipePlan plan;
    DeviceBuffer d_tab, d_e0, d_start, d_lrow, d_hc, d_stamps, d_pflags, d_spos, d_dtab;
    PipeModel view{};
    void upload(const PipePlan& p, uint32_t n, uint32_t S, hipStream_t s);
    void report_stamps(uint32_t nseq) const;  // diagnostic (SVH_PIPE_DEBUG): first sequence's waves
};

// Host tables of the on-chip _spec level-2 kernel (spec2.hip); ok == false when the model does
// not fit it (then level 2 streams dense products).
struct Spec2Plan {
    bool ok = false;
    bool prune = false;
    uint32_t R = 0, KL = 0, NHS = 0, nhs = 0, H = 0, NP = 0;
    std::vector<uint32_t> la, lb, thr, tcp, ha, hb, hrow;
    std::vector<float> lv, hv, amax;
};
Spec2Plan make_spec2_plan(const HostModel& hm);

struct DeviceSpec2Plan {
    Spec2Plan plan;
    DeviceBuffer d_la, d_lb, d_lv, d_thr, d_tcp, d_ha, d_hb, d_hv, d_hrow, d_amax, d_stamps;
    Spec2Model view{};
    void report_stamps(uint32_t nseq) const;  // diagnostic (SVH_SPEC2_DEBUG, -DSVH_SPEC2_DIAG builds)
    void upload(const Spec2Plan& p, const HostModel& hm, const float* d_emis, hipStream_t s);
};

// Pinned host staging buffer (grow-only).
template <class T>
struct Pinned {
    T* p = nullptr;
    size_t n = 0;
    Pinned() = default;
    Pinned(const Pinned&) = delete;
    Pinned& operator=(const Pinned&) = delete;
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
    T* reserve(size_t count) {
        if (count > n) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            n = 0;
            hip_check(hipHostMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault),
                      "hipHostMalloc");
            n = count;
        }
        return p;
    }
};

// Scratch of the pipelined kernel, owned by a batch (grow-only).
struct PipeScratchBuffers {
    DeviceBuffer d_ctr, d_done, d_part, d_gran, d_cons, d_viol, d_xcc;
    PipeScratch view{};
    uint64_t launches = 0;  // pipelined launches on this scratch (its device epoch counts the same)
    void ensure(uint32_t rows, uint32_t G, hipStream_t s);
    // before every launch: every kEpochSpan launches the granules, progress words and the epoch
    // counter are re-zeroed on s, so a granule tag (epoch modulo 0xFFFFF, pipe_common.h gtag)
    // never meets a stale granule of an earlier launch with the same residue
    void note_launch(hipStream_t s);
    static constexpr uint64_t kEpochSpan = 1ull << 19;
};

struct Model {
    std::mutex mu;
    int device = 0;
    int kernel_pref = SVH_KERNEL_AUTO;
    HostModel host;
    hipStream_t stream = nullptr;
    DeviceBandPlan band;             // chain kernel plan (scores-only runs of MSV-shaped models)
    DeviceBandPlan band_wide;        // chain plan for batches wider than the chip: streamed E,
                                     // 4 waves (more workgroups per CU), scores only
    uint32_t cu_count = 0;
    DevicePipePlan pipe;             // pipelined chain plan (latency path for small batches)
    uint32_t pipe_max_nseq = 0;      // AUTO: pipelined plan for scores-only batches of at most this many rows
    uint32_t pipe_max_nseq_paths = 0;  // ... for decoded-path batches
    uint32_t diag_max_nseq = 0;      // AUTO: the diagonal plan (diag.hip) for scores-only batches of at most this many rows
    // diagonal plan for a scores-only pass over nseq rows from observation 0 (nullptr: none)
    const DevicePipePlan* diag_for(uint32_t nseq) const;
    DevicePipePlan pipe_wide;        // wide pipelined plan (throughput path for batches that fill the chip)
    uint32_t pipew_min_nseq = 0;     // AUTO: wide pipelined plan for batches of at least this many rows
    DevicePlan fast_plan;            // fastest fused plan (may use uniform heavy rows)
    DevicePlan paths_plan_storage;   // term-by-term plan when fast_plan is uniform
    const DevicePlan* paths_plan = nullptr;
    DeviceBuffer d_gemis, d_gstart, d_rowptr, d_col, d_val, d_rowof;  // CSR (generic, _spec)
    // _spec products (level >= 3, or level 2 on models the on-chip kernel does not take)
    uint32_t spec_level = 0;
    uint32_t pstride = 0;
    DeviceBuffer d_mfold, d_products;
    // _spec level 2 on chip (spec2.hip): built by spec_build(2) unless SVH_SPEC_DENSE=1
    DeviceSpec2Plan spec2;
    bool spec2_on = false;
    // level 2 runs on the pipelined latency plan (pipe_l2.hip) with spec2_kernel as its exact
    // fallback: the model has both, every score >= 0, and the kernel preference allows the pipe
    bool pipe_l2_on() const;
    bool spec_dense = false;  // svh_model_opts.flags & SVH_MODEL_SPEC_DENSE

    Model(const HostModel& h, const svh_model_opts* opts);
    ~Model();
    CsrModel csr_view() const;
    // Fused plan to run (nullptr: generic kernel).
    const DevicePlan* plan_for(bool paths) const;
    // Chain plan to run for a pass over nseq sequences (nullptr: use plan_for(paths)).
    const DeviceBandPlan* band_for(bool paths, uint32_t nseq = 0) const;
    // Pipelined plan for a scores-only pass over nseq rows (nullptr: none).
    const DevicePipePlan* pipe_for(uint32_t nseq) const;
    // Pipelined plan for a decoded-path pass over nseq rows (nullptr: the chain / fused variant):
    // the latency plan, with the chain kernel's path variant as the fallback of flagged rows.
    const DevicePipePlan* pipe_paths_for(uint32_t nseq) const;
    void spec_build(uint32_t level, hipStream_t s);
    svh_model_info info(uint32_t nseq = 0, bool paths = false, uint32_t level = 0) const;
    // one pass of the step kernel the model plans for (chain, band, fused or generic)
    void launch_steps(const FusedBatch& b, bool paths, hipStream_t s) const;
};

struct Batch {
    Model* model;
    uint32_t nseq = 0;
    bool paths = false;
    std::vector<uint64_t> offsets;  // host copy of the caller's prefix offsets
    std::vector<uint32_t> lens;
    uint64_t total = 0;
    // inputs: one device arena (symbols, offset / begin / end tables, path offset tables),
    // uploaded from one pinned staging arena per load; the pointers are views into it
    DeviceBuffer d_in;
    Pinned<uint8_t> h_in;
    uint8_t* p_sym = nullptr;
    uint64_t* p_symoff = nullptr;
    uint32_t *p_begin = nullptr, *p_end = nullptr;
    uint64_t *p_pathoff = nullptr, *p_cmoff = nullptr, *p_hroff = nullptr, *p_ckoff = nullptr, *p_pmoff = nullptr,
             *p_proff = nullptr, *p_pcoff = nullptr, *p_fcoff = nullptr, *p_bpoff = nullptr;
    // results: one device arena {fault word (16 B) | best states | scores}: read() copies it once.
    // The fault word (FusedBatch::fault; kFault* bits) is written only by this batch's kernels
    // and read and cleared only by this batch.
    DeviceBuffer d_out;
    uint32_t* p_fault = nullptr;
    int64_t* p_best = nullptr;
    float* p_scores = nullptr;
    DeviceBuffer d_bp, d_paths;
    bool chain_paths = false;  // paths from the chain kernel's compact records (else fused / generic)
    DeviceBuffer d_cmask, d_hrec, d_ckpt;
    // paths on the pipelined plan (pipe.hip PATHS): its masks, partial records, checkpoints and F
    // checkpoints (the heavy records share d_hrec: the chain fallback writes only flagged rows)
    bool pipe_paths = false;
    DeviceBuffer d_pmask, d_prec, d_pck, d_fck;
    PipeScratchBuffers pipe;  // pipelined kernel scratch (sized for the rows of each launch)

    // _spec runs
    DeviceBuffer d_vbuf, d_nchunks, d_tbegin, d_vrow;
    DeviceBuffer d_l2viol;  // level 2 on the pipelined plan: rows whose speculation failed (spec2 re-runs them)
    bool l2_ran = false;    // the last run used it
    uint32_t spec_ready_level = 0;
    uint32_t max_chunks = 0;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    // SVH_BATCH_NO_TIMING: run() records no start / stop events (each event record is a marker on
    // the stream that the next kernel waits behind: ~3 us per record on MI355X); elapsed_ms() is then
    // unavailable and pipe_fallbacks() waits on the last run's stream instead
    bool timing = true;
    hipStream_t last_stream = nullptr;
    bool ran = false;

    // host tables of the last load (copied into h_in)
    Pinned<uint8_t> h_out;  // read(): the result arena and the paths land here in one sync
    std::vector<uint64_t> h_symoff, h_pathoff, h_bpoff, h_cmoff, h_hroff, h_ckoff;
    std::vector<uint64_t> h_pmoff, h_proff, h_pcoff, h_fcoff;

    Batch(Model* m, uint64_t nseq, const uint64_t* offsets, const uint64_t* symbols, uint32_t flags);
    Batch(Model* m, uint64_t nseq, const uint64_t* offsets, const uint8_t* symbols, uint32_t flags);
    // replace the sequences (same flags); uploads are asynchronous on s
    // (symbols from one packed array, sym64 or sym8, at `offsets`; or, with seqp, sequence q at
    //  seqp[q] with length offsets[q+1] - offsets[q])
    void load(uint64_t nseq, const uint64_t* offsets, const uint64_t* sym64, const uint8_t* sym8, hipStream_t s,
              const uint64_t* const* seqp = nullptr);
    ~Batch();
    void run(uint32_t level, hipStream_t s);
    void read(hipStream_t s, float* scores, int64_t* best, int32_t* paths);
    float elapsed_ms();
    // the latency plan's pass with no boundary exchange (FLOOR), ms per launch over `reps` (its own
    // scratch and outputs; svh_batch_step_floor_ms)
    float step_floor_ms(hipStream_t s, uint32_t reps);
    PipeScratchBuffers floor_scratch;
    DeviceBuffer d_floor_out;
    // rows of the last run that the pipelined kernel handed to the serial kernel (synchronous)
    // rows (nullable, nseq words): bit 0 the step pass re-ran the row, bit 1 the level-2 pass
    uint64_t pipe_fallbacks(uint32_t* rows = nullptr);
    bool pipe_ran = false;  // the last run used the pipelined kernel
    // opt-in time-parallel scores (segments of >= seg observations, probes of `probe`; see
    // runtime.cpp); synchronous; *fallbacks = segments that did not converge within the probe
    void run_time_parallel(uint32_t seg, uint32_t probe, float tol, hipStream_t s, uint64_t* fallbacks);
    // enqueue result copies (any pointer may be NULL) on s without waiting
    void read_async(hipStream_t s, float* scores, int64_t* best, int32_t* paths);
    // throws SVH_E_HIP if a bounded wait of this batch's last run gave up (waits on s; the word is
    // cleared on s when reported, so later runs are judged on their own)
    void check_fault(hipStream_t s);
    // diagnostics (svh_batch_debug_fault): mark the last run as if a bounded wait had given up
    void inject_fault(hipStream_t s);

  private:
    void init(uint32_t flags);
    void report_fault(uint32_t f, hipStream_t s);
};

}  // namespace svh
