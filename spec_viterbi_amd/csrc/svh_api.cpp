// extern "C" boundary (include/svh.h).  Every entry point catches everything, records a
// thread-local message and returns a status code: no exception crosses the ABI.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <mutex>
#include <new>
#include <string>

#include "HMM.h"
#include "data_reader.h"
#include "runtime.h"
#include "stream.h"
#include "svh.h"

struct svh_hmm {
    HMM hmm;
};
struct svh_ess {
    HMM::Emit_seq_vec_t seqs;
};
struct svh_model {
    std::unique_ptr<svh::Model> impl;
    // svh_viterbi's batches (scores only / with paths), kept between calls: their device buffers
    // only grow, so a one-shot call after the first allocates nothing and frees nothing (no
    // hipMalloc / hipFree device-wide syncs on the drop-in run_Viterbi path)
    std::mutex oneshot_mu;
    std::unique_ptr<svh::Batch> oneshot[2];
};
struct svh_batch {
    std::unique_ptr<svh::Batch> impl;
    svh_model* owner;
};
struct svh_reader {
    std::unique_ptr<svh::SeqReader> impl;
    std::vector<uint64_t> offsets;
    std::vector<uint8_t> symbols;
};

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

template <class F>
int guarded(F&& f) {
    try {
        g_last_error.clear();
        f();
        return SVH_OK;
    } catch (const svh::Error& e) {
        return fail(e.code, e.what());
    } catch (const std::bad_alloc&) {
        return fail(SVH_E_NOMEM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(SVH_E_INVALID, e.what());
    } catch (...) {
        return fail(SVH_E_INVALID, "unknown error");
    }
}

void require(bool ok, const char* what) {
    if (!ok) throw svh::Error(SVH_E_INVALID, what);
}

}  // namespace

extern "C" {

int svh_abi_version(void) { return SVH_ABI_VERSION; }

const char* svh_last_error(void) { return g_last_error.c_str(); }

int svh_device_count(int* count) {
    return guarded([&] {
        require(count != nullptr, "null count");
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
        *count = c;
    });
}

// ---- readers -------------------------------------------------------------------------------
int svh_hmm_read(const char* path, svh_hmm_t* out) {
    return guarded([&] {
        require(path && out, "null argument");
        *out = nullptr;
        if (!std::ifstream(path)) throw svh::Error(SVH_E_IO, std::string("cannot open ") + path);
        auto h = std::make_unique<svh_hmm>();
        h->hmm = read_HMM(path);
        *out = h.release();
    });
}

int svh_hmm_dims(svh_hmm_t h, uint64_t* n, uint64_t* S, uint64_t* nstart, uint64_t* ntrans) {
    return guarded([&] {
        require(h != nullptr, "null handle");
        if (n) *n = h->hmm.states_num;
        if (S) *S = h->hmm.emit_num;
        if (nstart) *nstart = h->hmm.start_probabilities.size();
        if (ntrans) *ntrans = h->hmm.trans_probs.size();
    });
}

int svh_hmm_copy(svh_hmm_t h, uint64_t* start_cols, float* start_vals, float* emissions,
                 uint64_t* trans_src, uint64_t* trans_dst, float* trans_prob) {
    return guarded([&] {
        require(h != nullptr, "null handle");
        const HMM& m = h->hmm;
        for (size_t i = 0; i < m.start_probabilities.size(); ++i) {
            if (start_cols) start_cols[i] = m.start_probabilities_cols[i];
            if (start_vals) start_vals[i] = m.start_probabilities[i];
        }
        if (emissions)
            for (size_t o = 0; o < m.emissions.size(); ++o)
                for (size_t j = 0; j < m.emissions[o].size(); ++j)
                    emissions[o * m.states_num + j] = m.emissions[o][j];
        for (size_t e = 0; e < m.trans_probs.size(); ++e) {
            if (trans_src) trans_src[e] = m.trans_rows[e];
            if (trans_dst) trans_dst[e] = m.trans_cols[e];
            if (trans_prob) trans_prob[e] = m.trans_probs[e];
        }
    });
}

void svh_hmm_free(svh_hmm_t h) { delete h; }

int svh_ess_read(const char* path, svh_ess_t* out) {
    return guarded([&] {
        require(path && out, "null argument");
        *out = nullptr;
        if (!std::ifstream(path)) throw svh::Error(SVH_E_IO, std::string("cannot open ") + path);
        auto e = std::make_unique<svh_ess>();
        e->seqs = read_emit_seq(path);
        *out = e.release();
    });
}

int svh_ess_dims(svh_ess_t e, uint64_t* nseq, uint64_t* total) {
    return guarded([&] {
        require(e != nullptr, "null handle");
        uint64_t t = 0;
        for (const auto& s : e->seqs) t += s.size();
        if (nseq) *nseq = e->seqs.size();
        if (total) *total = t;
    });
}

int svh_ess_copy(svh_ess_t e, uint64_t* offsets, uint64_t* symbols) {
    return guarded([&] {
        require(e != nullptr, "null handle");
        uint64_t t = 0;
        for (size_t q = 0; q < e->seqs.size(); ++q) {
            if (offsets) offsets[q] = t;
            for (size_t i = 0; i < e->seqs[q].size(); ++i)
                if (symbols) symbols[t + i] = e->seqs[q][i];
            t += e->seqs[q].size();
        }
        if (offsets) offsets[e->seqs.size()] = t;
    });
}

void svh_ess_free(svh_ess_t e) { delete e; }

// ---- model ---------------------------------------------------------------------------------
int svh_model_create(uint64_t n, uint64_t S, uint64_t nstart, const uint64_t* start_cols,
                     const float* start_vals, const float* emissions, uint64_t ntrans,
                     const uint64_t* trans_src, const uint64_t* trans_dst,
                     const float* trans_prob, const svh_model_opts* opts, svh_model_t* out) {
    return guarded([&] {
        require(out != nullptr, "null output handle");
        *out = nullptr;
        svh::HostModel h = svh::build_host_model(n, S, nstart, start_cols, start_vals, emissions,
                                                 ntrans, trans_src, trans_dst, trans_prob);
        auto m = std::make_unique<svh_model>();
        m->impl = std::make_unique<svh::Model>(h, opts);
        *out = m.release();
    });
}

int svh_model_destroy(svh_model_t m) {
    return guarded([&] { delete m; });
}

int svh_model_get_info(svh_model_t m, svh_model_info* info) {
    return guarded([&] {
        require(m && info, "null argument");
        *info = m->impl->info();
    });
}

int svh_spec_build(svh_model_t m, uint32_t level, void* stream) {
    return guarded([&] {
        require(m != nullptr, "null model");
        m->impl->spec_build(level, static_cast<hipStream_t>(stream));
    });
}

// ---- batches -------------------------------------------------------------------------------
int svh_batch_create(svh_model_t m, uint64_t nseq, const uint64_t* offsets,
                     const uint64_t* symbols, uint32_t flags, svh_batch_t* out) {
    return guarded([&] {
        require(m && out, "null argument");
        *out = nullptr;
        auto b = std::make_unique<svh_batch>();
        b->owner = m;
        b->impl = std::make_unique<svh::Batch>(m->impl.get(), nseq, offsets, symbols, flags);
        *out = b.release();
    });
}

int svh_batch_create_u8(svh_model_t m, uint64_t nseq, const uint64_t* offsets, const uint8_t* symbols,
                        uint32_t flags, svh_batch_t* out) {
    return guarded([&] {
        require(m && out, "null argument");
        *out = nullptr;
        auto b = std::make_unique<svh_batch>();
        b->owner = m;
        b->impl = std::make_unique<svh::Batch>(m->impl.get(), nseq, offsets, symbols, flags);
        *out = b.release();
    });
}

int svh_batch_run(svh_batch_t b, uint32_t level, void* stream) {
    return guarded([&] {
        require(b != nullptr, "null batch");
        b->impl->run(level, static_cast<hipStream_t>(stream));
    });
}

int svh_batch_run_time_parallel(svh_batch_t b, uint32_t seg_len, uint32_t probe_len, float rel_tol,
                                void* stream, uint64_t* fallbacks) {
    return guarded([&] {
        require(b != nullptr, "null batch");
        b->impl->run_time_parallel(seg_len, probe_len, rel_tol, static_cast<hipStream_t>(stream), fallbacks);
    });
}

int svh_host_alloc(size_t bytes, void** out) {
    return guarded([&] {
        require(out != nullptr, "null argument");
        *out = nullptr;
        svh::hip_check(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault), "hipHostMalloc");
    });
}

int svh_host_free(void* p) {
    return guarded([&] {
        if (p) svh::hip_check(hipHostFree(p), "hipHostFree");
    });
}

int svh_batch_read(svh_batch_t b, void* stream, float* scores, int64_t* best_state,
                   int32_t* paths) {
    return guarded([&] {
        require(b != nullptr, "null batch");
        b->impl->read(static_cast<hipStream_t>(stream), scores, best_state, paths);
    });
}

int svh_batch_device_results(svh_batch_t b, float** scores, int64_t** best_state) {
    return guarded([&] {
        require(b != nullptr, "null batch");
        if (scores) *scores = b->impl->p_scores;
        if (best_state) *best_state = b->impl->p_best;
    });
}

int svh_batch_elapsed_ms(svh_batch_t b, float* ms) {
    return guarded([&] {
        require(b && ms, "null argument");
        *ms = b->impl->elapsed_ms();
    });
}

int svh_batch_step_floor_ms(svh_batch_t b, void* stream, uint32_t reps, float* ms) {
    return guarded([&] {
        require(b && ms && reps > 0, "null argument or reps == 0");
        *ms = b->impl->step_floor_ms(static_cast<hipStream_t>(stream), reps);
    });
}

int svh_batch_fallback_rows(svh_batch_t b, uint32_t* flags) {
    return guarded([&] {
        require(b && flags, "null argument");
        (void)b->impl->pipe_fallbacks(flags);
    });
}

int svh_batch_fallbacks(svh_batch_t b, uint64_t* rows) {
    return guarded([&] {
        require(b && rows, "null argument");
        *rows = b->impl->pipe_fallbacks();
    });
}

int svh_pipe_variant_built(int32_t slots, int32_t waves, int32_t table_mode, int32_t* built) {
    return guarded([&] {
        require(built != nullptr, "null argument");
        bool ok = false;
        if (table_mode == 0) ok = svh::pipe_supported(slots, waves, false);
        else ok = slots == 2 && waves == 4 && svh::pipe_tm_supported(table_mode);
        *built = ok ? 1 : 0;
    });
}

int svh_batch_debug_fault(svh_batch_t b, void* stream) {
    return guarded([&] {
        require(b != nullptr, "null batch");
        b->impl->inject_fault(static_cast<hipStream_t>(stream));
    });
}

int svh_batch_plan(svh_batch_t b, uint32_t level, svh_model_info* info) {
    return guarded([&] {
        require(b && info, "null argument");
        *info = b->impl->model->info(b->impl->nseq, b->impl->paths, level);
    });
}

int svh_batch_destroy(svh_batch_t b) {
    return guarded([&] { delete b; });
}

namespace {
// svh_viterbi*: the model's kept batch (scores only / with paths), reloaded from the caller's
// symbols in whichever form they come, then one run and one read (throws; callers guard)
void oneshot(svh_model_t m, uint32_t level, uint64_t nseq, const uint64_t* offsets, const uint64_t* sym64,
             const uint8_t* sym8, const uint64_t* const* seqp, float* scores, int64_t* best_state, int32_t* paths) {
    require(m != nullptr, "null model");
    require(offsets && (sym64 || sym8 || seqp), "null offsets/symbols");
    std::lock_guard<std::mutex> lock(m->oneshot_mu);
    std::unique_ptr<svh::Batch>& b = m->oneshot[paths ? 1 : 0];
    if (!b) {  // created once with a one-symbol placeholder; the load below replaces it
        static const uint64_t one[2] = {0, 1};
        static const uint8_t zero = 0;
        b = std::make_unique<svh::Batch>(m->impl.get(), 1, one, &zero, paths ? SVH_BATCH_PATHS : 0u);
    }
    // SVH_TRACE_ONESHOT=1 (diagnostics): host microseconds of each phase and the GPU time from the
    // call's first enqueue to the run's start event, on stderr
    static const bool trace = std::getenv("SVH_TRACE_ONESHOT") && std::atoi(std::getenv("SVH_TRACE_ONESHOT"));
    if (!trace) {
        b->load(nseq, offsets, sym64, sym8, m->impl->stream, seqp);
        b->run(level, nullptr);
        b->read(nullptr, scores, best_state, paths);
        return;
    }
    using clk = std::chrono::steady_clock;
    hipEvent_t e0;
    (void)hipEventCreate(&e0);
    const auto t0 = clk::now();
    (void)hipEventRecord(e0, m->impl->stream);
    b->load(nseq, offsets, sym64, sym8, m->impl->stream, seqp);
    const auto t1 = clk::now();
    b->run(level, nullptr);
    const auto t2 = clk::now();
    b->read(nullptr, scores, best_state, paths);
    const auto t3 = clk::now();
    float upload_ms = 0.0f, kernel_ms = 0.0f;
    (void)hipEventElapsedTime(&upload_ms, e0, b->ev_start);
    (void)hipEventElapsedTime(&kernel_ms, b->ev_start, b->ev_stop);
    (void)hipEventDestroy(e0);
    auto us = [](clk::time_point a, clk::time_point c) { return std::chrono::duration<double, std::micro>(c - a).count(); };
    std::fprintf(stderr, "oneshot trace (us): load %.1f run-enqueue %.1f read %.1f total %.1f | gpu: upload-to-run-start %.1f "
                 "run %.1f\n", us(t0, t1), us(t1, t2), us(t2, t3), us(t0, t3), upload_ms * 1e3, kernel_ms * 1e3);
}
}  // namespace

int svh_viterbi(svh_model_t m, uint32_t level, uint64_t nseq, const uint64_t* offsets,
                const uint64_t* symbols, float* scores, int64_t* best_state, int32_t* paths) {
    return guarded([&] { oneshot(m, level, nseq, offsets, symbols, nullptr, nullptr, scores, best_state, paths); });
}

int svh_viterbi_u8(svh_model_t m, uint32_t level, uint64_t nseq, const uint64_t* offsets,
                   const uint8_t* symbols, float* scores, int64_t* best_state, int32_t* paths) {
    return guarded([&] { oneshot(m, level, nseq, offsets, nullptr, symbols, nullptr, scores, best_state, paths); });
}

int svh_viterbi_seqs(svh_model_t m, uint32_t level, uint64_t nseq, const uint64_t* const* seqs,
                     const uint64_t* lens, float* scores, int64_t* best_state, int32_t* paths) {
    return guarded([&] {
        require(seqs && lens, "null sequences/lengths");
        std::vector<uint64_t> offs(nseq + 1, 0);
        for (uint64_t q = 0; q < nseq; ++q) offs[q + 1] = offs[q] + lens[q];
        oneshot(m, level, nseq, offs.data(), nullptr, nullptr, seqs, scores, best_state, paths);
    });
}

// ---- streaming ingestion -----------------------------------------------------------------
int svh_reader_open(const char* path, int format, svh_reader_t* out) {
    return guarded([&] {
        require(path && out, "null argument");
        *out = nullptr;
        auto r = std::make_unique<svh_reader>();
        r->impl = std::make_unique<svh::SeqReader>(path, format);
        *out = r.release();
    });
}

int svh_reader_next(svh_reader_t r, uint64_t max_seqs, uint64_t max_symbols, uint64_t* nseq,
                    const uint64_t** offsets, const uint8_t** symbols) {
    return guarded([&] {
        require(r && nseq, "null argument");
        *nseq = 0;
        if (!r->impl->next(max_seqs, max_symbols, r->offsets, r->symbols)) r->offsets.assign(1, 0);
        *nseq = r->offsets.size() - 1;
        if (offsets) *offsets = r->offsets.data();
        if (symbols) *symbols = r->symbols.data();
    });
}

void svh_reader_close(svh_reader_t r) { delete r; }

int svh_decode_file(svh_model_t m, const char* path, int format, uint32_t level, uint32_t flags,
                    uint64_t max_seqs, uint64_t max_symbols, svh_result_fn fn, void* user,
                    uint64_t* nseq_total) {
    return guarded([&] {
        require(m && path && fn, "null argument");
        if (nseq_total) *nseq_total = 0;
        const uint64_t n = svh::decode_file(m->impl.get(), path, format, level, flags, max_seqs, max_symbols, fn, user);
        if (nseq_total) *nseq_total = n;
    });
}

}  // extern "C"
