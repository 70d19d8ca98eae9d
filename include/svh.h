/*
 * svh.h -- C ABI of the MI355X (gfx950) Viterbi engine, libspec_viterbi_hip.so.
 *
 * This is the drop-in boundary for the reference's hot path.  Every entry point names the
 * reference interface it replaces (paths relative to the IvanTyulyandin/Spec_Viterbi checkout):
 *
 *   svh_hmm_read / svh_hmm_*        read_HMM                        Viterbi_impl/data_reader.h:8
 *   svh_ess_read / svh_ess_*        read_emit_seq                   Viterbi_impl/data_reader.h:11
 *   svh_model_create                per-call model setup of GraphBLAS_impl::run_Viterbi
 *                                   (GraphBLAS_impl.cpp:9-54), done once and kept in HBM
 *   svh_viterbi / svh_batch_*       Viterbi_impl::run_Viterbi       Viterbi_impl/Viterbi_impl.h:8-9
 *                                   (batched: one call = many sequences)
 *   svh_spec_build                  Viterbi_spec_impl::spec_with    Viterbi_impl/Viterbi_spec_impl.h:11
 *   svh_viterbi(level >= 1)         Viterbi_spec_impl::run_Viterbi_spec  Viterbi_spec_impl.h:13-14
 *
 * Conventions: plain pointers and sizes, no C++ or torch types; every call returns an int status
 * (SVH_OK == 0); svh_last_error() gives a thread-local message for the last failure; host
 * buffers are caller-owned and only borrowed during the call; indices and symbols are uint64_t
 * (the reference's size_t HMM::Index_t / HMM::Emit_t); scores are -log2 probabilities (fp32,
 * +inf = impossible), bit-identical to GraphBLAS_impl.  Handles are thread-safe.
 * A `stream` argument is a hipStream_t (NULL = the handle's own stream).
 */
#ifndef SPEC_VITERBI_SVH_H
#define SPEC_VITERBI_SVH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVH_ABI_VERSION 4  /* 2: svh_model_info pipe_* fields, SVH_KERNEL_PIPE, svh_batch_fallbacks;
                              3: pipe_max_nseq_paths, SVH_KERNEL_SPEC2_PIPE, SVH_BATCH_NO_TIMING;
                              4: SVH_KERNEL_DIAG, svh_model_info diag_* fields */

enum {
    SVH_OK = 0,
    SVH_E_INVALID = -1,     /* bad argument (null pointer, empty sequence, ...) */
    SVH_E_RANGE = -2,       /* state index or symbol out of range */
    SVH_E_NOMEM = -3,       /* host or device allocation failed */
    SVH_E_HIP = -4,         /* HIP runtime error (no device, launch failure, ...) */
    SVH_E_UNSUPPORTED = -5, /* valid request this build does not implement */
    SVH_E_STATE = -6,       /* e.g. run at spec level L before svh_spec_build(L) */
    SVH_E_IO = -7           /* file could not be opened / parsed */
};

typedef struct svh_hmm* svh_hmm_t;
typedef struct svh_ess* svh_ess_t;
typedef struct svh_model* svh_model_t;
typedef struct svh_batch* svh_batch_t;

int svh_abi_version(void);
const char* svh_last_error(void);
int svh_device_count(int* count);

/* ---- readers (host; same parse and error semantics as data_reader.cpp) ------------------ */
int svh_hmm_read(const char* path, svh_hmm_t* out);
int svh_hmm_dims(svh_hmm_t h, uint64_t* n, uint64_t* S, uint64_t* nstart, uint64_t* ntrans);
int svh_hmm_copy(svh_hmm_t h, uint64_t* start_cols, float* start_vals, float* emissions,
                 uint64_t* trans_src, uint64_t* trans_dst, float* trans_prob);
void svh_hmm_free(svh_hmm_t h);
int svh_ess_read(const char* path, svh_ess_t* out);
int svh_ess_dims(svh_ess_t e, uint64_t* nseq, uint64_t* total_symbols);
int svh_ess_copy(svh_ess_t e, uint64_t* offsets /* nseq + 1 */, uint64_t* symbols);
void svh_ess_free(svh_ess_t e);

/* ---- model: HMM resident in HBM -------------------------------------------------------- */
/* AUTO: for scores-only passes over chain-shaped (MSV) models the barrier-free register chain
 * kernel (CHAIN, emit_num <= 32, <= 2560 light states), else the barrier chain kernel (BAND);
 * otherwise the fused kernel, else the generic one.  BAND / CHAIN force that kernel (error if the
 * model does not qualify).  Path runs use the chain kernel's decoded-path variant when the model
 * is chain-shaped with at most one heavy row feeding the light rows (every reference .chmm), else
 * the fused (or generic) kernel with 16-bit backpointers. */
enum { SVH_KERNEL_AUTO = 0, SVH_KERNEL_FUSED = 1, SVH_KERNEL_GENERIC = 2, SVH_KERNEL_BAND = 3,
       SVH_KERNEL_CHAIN = 4, SVH_KERNEL_PIPE = 5, SVH_KERNEL_PIPE_WIDE = 6, SVH_KERNEL_SPEC2 = 7,
       SVH_KERNEL_SPEC2_PIPE = 8, SVH_KERNEL_DIAG = 9 };
/* PIPE: the pipelined chain kernel (MSV-shaped models whose feeder row N takes terms only from
 * the light rows and itself): a sequence's states are split over many waves and CUs; N's light
 * term is speculated away and checked exactly at every observation, and a sequence that fails
 * the check is re-run exactly (scores: inside the same launch by the row's combining workgroup;
 * paths and the wide plan: by the serial chain kernel) -- the same results either way.  AUTO uses it for
 * scores-only passes over batches too small to fill the chip with the chain kernel.
 * PIPE_WIDE: the same recurrence with one block of states per workgroup and one sequence per wave
 * (the block's table in LDS, shared by the waves): the throughput plan AUTO uses for wider
 * batches.
 * SPEC2 (reported by svh_batch_plan only, not selectable): _spec level 2 evaluated on chip from
 * the folded sparse matrices, one workgroup per sequence (spec2.hip); the odd last observation of
 * a sequence runs on the step kernels.
 * SPEC2_PIPE (reported by svh_batch_plan only): _spec level 2 on the pipelined latency plan
 * (pipe_l2.hip: every chunk of every row in one launch, the light term of N and its two-hop terms
 * speculated away and checked exactly, flagged rows re-run by spec2.hip); AUTO and PIPE use it for
 * MSV-shaped models whose scores are all >= 0.
 * DIAG: the pipelined plan's recurrence with every lane on an anti-diagonal of the (state,
 * observation) grid: a state's chain input is the lane's own previous score, so no wave waits for
 * another (diag.hip).  Scores-only passes from the first observation; AUTO uses it for the batches
 * the latency plan used to take (svh_model_info.diag_max_nseq); selecting it runs every scores-only
 * pass of the model on it (decoded paths and the _spec tail use the chain kernel). */

typedef struct {
    int32_t device;      /* HIP device ordinal; -1 = the caller's current device */
    int32_t kernel;      /* SVH_KERNEL_* */
    int32_t max_threads; /* workgroup size cap (multiple of 64, <= 1024; the fused kernel caps at
                            512); 0 = each kernel's default */
    int32_t flags;       /* SVH_MODEL_* bits (0: defaults) */
} svh_model_opts;

/* svh_model_opts.flags: _spec level 2 streams the dense products (the path used for level >= 3)
 * instead of evaluating each chunk from the folded sparse matrices on chip (A/B and tests; the
 * results are identical) */
#define SVH_MODEL_SPEC_DENSE 1

/* emissions: S x n, symbol-major (HMM::emissions[symbol][state]); transitions as COO
 * src -> dst (HMM::trans_rows / trans_cols / trans_probs); duplicates: first one wins
 * (GrB_FIRST_FP32, GraphBLAS_impl.cpp:42-44). */
int svh_model_create(uint64_t n, uint64_t S, uint64_t nstart, const uint64_t* start_cols,
                     const float* start_vals, const float* emissions, uint64_t ntrans,
                     const uint64_t* trans_src, const uint64_t* trans_dst,
                     const float* trans_prob, const svh_model_opts* opts, svh_model_t* out);
int svh_model_destroy(svh_model_t m);

typedef struct {
    int32_t kernel;        /* SVH_KERNEL_CHAIN, _BAND, _FUSED or _GENERIC (scores-only runs) */
    int32_t family;        /* fused family id (0: R2 uniform-heavy, 1: R2, 2: R4, 3: R8, 4: R16) */
    int32_t threads;       /* workgroup size */
    int32_t slots;         /* states per thread */
    int32_t light_terms;   /* R */
    int32_t heavy_rows;    /* H */
    int32_t heavy_uniform; /* 1 if heavy rows use the shared dominant-weight reduction */
    int32_t device;
    uint64_t n, S, nnz;
    uint64_t lds_bytes;
    uint64_t spec_level;   /* level of the products built by svh_spec_build (0/1: none needed) */
    uint64_t spec_bytes;   /* HBM held by the products */
    int32_t paths_kernel;  /* kernel of decoded-path runs (SVH_KERNEL_CHAIN, _FUSED or _GENERIC) */
    int32_t wide_threads;  /* chain plan for batches of more sequences than CUs (streamed E, more
                              workgroups per CU): its threads per workgroup, 0 = none */
    int32_t wide_slots;    /* ... and its states per thread */
    uint32_t cu_count;     /* CUs of the model's device: batches of more sequences switch plans */
    int32_t pipe_slots;    /* pipelined plan (SVH_KERNEL_PIPE): states per lane, 0 = none */
    int32_t pipe_waves;    /* ... waves per workgroup */
    int32_t pipe_groups;   /* ... workgroups per sequence */
    uint32_t pipe_max_nseq; /* AUTO runs the pipelined plan for batches of at most this many sequences */
    int32_t pipew_slots;   /* wide pipelined plan (SVH_KERNEL_PIPE_WIDE): states per lane, 0 = none */
    int32_t pipew_waves;   /* ... sequences (waves) per workgroup */
    int32_t pipew_blocks;  /* ... workgroups per sequence */
    uint32_t pipew_min_nseq; /* AUTO runs it for batches of at least this many sequences */
    uint32_t pipe_max_nseq_paths; /* ... the latency plan's bound for decoded-path batches (one
                                     workgroup per CU; pipe_max_nseq allows two for scores; the
                                     SVH_PIPE_MAX_NSEQ override applies to scores only) */
    int32_t diag_ranges;   /* diagonal plan (SVH_KERNEL_DIAG): ranges of 64 diagonals per sequence, 0 = none */
    uint32_t diag_max_nseq; /* AUTO runs it for scores-only batches of at most this many sequences */
} svh_model_info;
/* The model's plan for a one-sequence scores-only run (kernel/threads/slots describe it). */
int svh_model_get_info(svh_model_t m, svh_model_info* info);

/* ---- _spec: precomputed products of `level` consecutive observations ------------------- */
/* level <= 1: nothing to precompute (the fused kernel folds diag(E_o) (x) T^T on the fly,
 * bit-identical to GraphBLAS_spec_impl level 1).  level >= 2: builds the S^level dense
 * n x n products H[(k1..kL)] = M_kL (x) ... (x) M_k1 in HBM (GraphBLAS_spec_impl.cpp:15-36,
 * 146-181).  Replaces any previous products. */
int svh_spec_build(svh_model_t m, uint32_t level, void* stream);

/* ---- batches: sequences resident in HBM ------------------------------------------------ */
/* SVH_BATCH_PATHS: decoded paths.  SVH_BATCH_NO_TIMING: svh_batch_run records no start / stop
 * events on the stream (svh_batch_elapsed_ms then fails with SVH_E_STATE); for callers that time
 * the stream themselves -- each event record is a marker the next kernel waits behind. */
enum { SVH_BATCH_PATHS = 1, SVH_BATCH_NO_TIMING = 2 };

/* offsets: nseq + 1 prefix offsets into symbols; every sequence must be non-empty. */
int svh_batch_create(svh_model_t m, uint64_t nseq, const uint64_t* offsets,
                     const uint64_t* symbols, uint32_t flags, svh_batch_t* out);
/* Enqueue one pass over the batch on `stream` (asynchronous).  level 0 = GraphBLAS_impl
 * semantics; level 1 = identical; level >= 2 = GraphBLAS_spec_impl(level) semantics (needs
 * svh_spec_build(level)).  Paths need level <= 1 and SVH_BATCH_PATHS. */
int svh_batch_run(svh_batch_t b, uint32_t level, void* stream);
/* Opt-in time-parallel pass (scores only, level 0).  Sequences longer than
 * 2*seg_len are cut into equal segments of >= seg_len observations that all run at once from
 * guesses: a light guess (zeros, heavy rows +inf) and, for chain/band models, one unit vector per
 * heavy row.  Segment k is then fixed up on the device from the corrected end v of k-1: the
 * heavy-row runs shifted by v's heavy scores are exact by (min,+)-linearity, and a probe of
 * probe_len observations from v's light part is compared with the light guess's probe -- if they
 * differ by a constant (within rel_tol of the best score) wherever the light part is not already
 * dominated by the heavy-row terms, the light guess's end plus that constant is taken, else the
 * rest of the segment is re-run exactly.  Scores match the serial pass up to rounding (not
 * bit-exact); rel_tol < 0 re-runs every segment (bit-exact, for verification).  *fallbacks
 * (nullable) = segments that were re-run.  Synchronous (one host wait at the end). */
int svh_batch_run_time_parallel(svh_batch_t b, uint32_t seg_len, uint32_t probe_len, float rel_tol,
                                void* stream, uint64_t* fallbacks);
/* Synchronise `stream` and copy results to host (any pointer may be NULL).  Scores and paths
 * buffers from svh_host_alloc (pinned) are written by the DMA engine directly; pageable buffers
 * are filled from the batch's pinned staging after the copy. */
int svh_batch_read(svh_batch_t b, void* stream, float* scores /* nseq * n */,
                   int64_t* best_state /* nseq */, int32_t* paths /* offsets[nseq] */);
/* Page-locked host memory for result buffers (svh_batch_read / svh_viterbi* write into it without
 * a staging copy).  svh_host_free releases it. */
int svh_host_alloc(size_t bytes, void** out);
int svh_host_free(void* p);
/* Device pointers of the results (for device-side gathers). */
int svh_batch_device_results(svh_batch_t b, float** scores, int64_t** best_state);
/* Milliseconds between the start and stop events of the last svh_batch_run (synchronises). */
int svh_batch_elapsed_ms(svh_batch_t b, float* ms);
/* Measurement (the latency plan's roofline): milliseconds per launch, mean of `reps`,
 * of the batch's pipelined latency pass with every boundary exchange removed -- each wave sweeps
 * its block as the first block does, with no input from its neighbours and no waits -- so the
 * launch takes the step's own per-observation time plus the prologue.  Its scores go to a scratch
 * buffer (they are not the batch's results, which this call leaves untouched).  SVH_E_UNSUPPORTED
 * unless the batch's scores-only plan is the pipelined latency plan at its default table mode.
 * Synchronous. */
int svh_batch_step_floor_ms(svh_batch_t b, void* stream, uint32_t reps, float* ms);
/* The plan svh_batch_run(level) launches for this batch (its sequence count and paths flag
 * decide between the narrow and the wide chain plan): kernel/threads/slots of the model info. */
int svh_batch_plan(svh_batch_t b, uint32_t level, svh_model_info* info);
/* Rows of the last run whose pipelined pass (SVH_KERNEL_PIPE, _PIPE_WIDE, _SPEC2_PIPE) failed its
 * speculation check and were re-run exactly (in the same launch, by the serial chain kernel, or at
 * level 2 by the on-chip chunk kernel; results are identical either way); 0 if the last run did
 * not use a pipelined kernel.  Waits for the run. */
int svh_batch_fallbacks(svh_batch_t b, uint64_t* rows);
/* The same per row: flags[q] (nseq words) bit 0 = the step pass re-ran row q, bit 1 = the _spec
 * level-2 pass on the pipelined plan handed it to the on-chip chunk kernel.  Waits for the run. */
int svh_batch_fallback_rows(svh_batch_t b, uint32_t* flags);
/* Whether this build holds the pipelined latency kernel at `slots` x `waves` with step table mode
 * `table_mode` (pipe_kernel.h TM; SVH_PIPE_SM / SVH_PIPE_WAVES / SVH_PIPE_TM select them).  The
 * default build holds the geometry and modes AUTO plans (2 x 4; TM 4, and TM 0 for alphabets of
 * more than 20 symbols); the others are A/B builds' (-DSVH_PIPE_AB_ALL).  *built = 1 or 0. */
int svh_pipe_variant_built(int32_t slots, int32_t waves, int32_t table_mode, int32_t* built);
int svh_batch_destroy(svh_batch_t b);
/* Diagnostics: mark the batch's last run (enqueued on `stream`) as if one of its bounded waits
 * had given up, so its next svh_batch_read fails with SVH_E_HIP.  Every batch has a fault word of
 * its own that only its runs set and only its reads report and clear (tests of that isolation). */
int svh_batch_debug_fault(svh_batch_t b, void* stream);

/* Batch from uint8 symbols (the device format; e.g. straight from svh_reader_next). */
int svh_batch_create_u8(svh_model_t m, uint64_t nseq, const uint64_t* offsets,
                        const uint8_t* symbols, uint32_t flags, svh_batch_t* out);

/* ---- streaming ingestion (the input side of the path) ------------------ */
/* .ess: read_emit_seq semantics (data_reader.cpp:93-134).  FASTA: fasta_to_ess.py semantics
 * (ess_files/fasta_to_ess.py:3-45): residues ACDEFGHIKLMNPQRSTVWY -> 0..19, X -> 0, lines
 * stripped, '>' starts a sequence, an empty line or another residue is an error.  AUTO: by
 * extension (.fasta/.fa/.faa/.fas, .ess), else by a leading '>'. */
enum { SVH_FORMAT_AUTO = 0, SVH_FORMAT_ESS = 1, SVH_FORMAT_FASTA = 2 };
typedef struct svh_reader* svh_reader_t;
int svh_reader_open(const char* path, int format, svh_reader_t* out);
/* The next chunk of whole sequences: at most max_seqs and at most max_symbols symbols in total
 * (a single longer sequence comes alone).  *nseq == 0 at the end.  offsets (nseq + 1, from 0) and
 * symbols point into reader-owned memory valid until the next call. */
int svh_reader_next(svh_reader_t r, uint64_t max_seqs, uint64_t max_symbols, uint64_t* nseq,
                    const uint64_t** offsets, const uint8_t** symbols);
void svh_reader_close(svh_reader_t r);

/* Results of one chunk of svh_decode_file (host memory valid during the call; paths NULL
 * unless SVH_BATCH_PATHS).  Return non-zero to stop. */
typedef int (*svh_result_fn)(void* user, uint64_t first_seq, uint64_t nseq, const uint64_t* offsets,
                             const float* scores, const int64_t* best_state, const int32_t* paths);
/* Decode a whole file chunk by chunk (chunks as svh_reader_next): parsing runs on a host thread
 * ahead of the GPU, chunk k's kernels overlap chunk k-1's result copies and hand-off, in file
 * order on the calling thread.  *nseq_total (nullable) = sequences decoded.  On a parse error the
 * chunks before it have been delivered. */
int svh_decode_file(svh_model_t m, const char* path, int format, uint32_t level, uint32_t flags,
                    uint64_t max_seqs, uint64_t max_symbols, svh_result_fn fn, void* user,
                    uint64_t* nseq_total);

/* ---- one-shot convenience: upload, run, download --------------------------------------- */
/* The model keeps the batch it used (one for scores only, one with paths) and reloads it on the
 * next call: device buffers only grow, so repeated calls allocate and free nothing.  Calls on one
 * model are serialised. */
int svh_viterbi(svh_model_t m, uint32_t level, uint64_t nseq, const uint64_t* offsets,
                const uint64_t* symbols, float* scores, int64_t* best_state, int32_t* paths);
/* The same from packed uint8 symbols (the device format: e.g. svh_reader_next's output), */
int svh_viterbi_u8(svh_model_t m, uint32_t level, uint64_t nseq, const uint64_t* offsets,
                   const uint8_t* symbols, float* scores, int64_t* best_state, int32_t* paths);
/* ... and from nseq separate symbol arrays (seqs[q], lens[q] symbols each: the reference's
 * HMM::Emit_seq_vec_t, a vector of vectors, or a list of arrays) without the caller flattening
 * them: each is narrowed straight into the pinned upload.  Paths (when requested) are written
 * back to back in sequence order. */
int svh_viterbi_seqs(svh_model_t m, uint32_t level, uint64_t nseq, const uint64_t* const* seqs,
                     const uint64_t* lens, float* scores, int64_t* best_state, int32_t* paths);

#ifdef __cplusplus
}
#endif

#endif
