/*
 * viterbi_oracle.h -- CPU restatement of the reference's GraphBLAS Viterbi semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (spec_viterbi_amd/, include/) may link,
 * load or call this code; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * use it, as the checker / baseline.
 *
 * Restates (file:line relative to the reference checkout):
 *   - GraphBLAS_impl::run_Viterbi            Viterbi_impl/GraphBLAS_impl.cpp:4-93
 *       v0[j]  = fl(E[s0][j] + start[j])                                   (:59)
 *       v'[j]  = min_k fl( fl(E[o][j] + T^T[j][k]) + v[k] )                (:64-73)
 *     with T^T built by GrB_Matrix_build(..., GrB_FIRST_FP32) (:38-45; first duplicate wins),
 *     min over an empty / all-absent row = absent = +inf (GraphBLAS_helper.cpp:65-68).
 *   - GraphBLAS_spec_impl                     Viterbi_impl/GraphBLAS_spec_impl.cpp
 *       M_o = diag(E_o) (x) T^T                (:146-161)
 *       H[(k..., i)] = M_i (x) H[(k...)]       (add_level, :15-36; level-1 H = M_o, :168-181)
 *       run: level-sized chunks v' = H[key] (x) v, tail v' = M_o (x) v   (:50-97)
 *   - Decoded-path extension (not in the reference): per-step argmin
 *     backpointers, ties broken toward the lowest predecessor index, final state = lowest index
 *     of the minimum final score.
 *
 * Parity pinning: the reference's GraphBLAS backend cannot be built here (SuiteSparse:GraphBLAS
 * is neither installed nor vendored).  This restatement is pinned by the reference's own golden
 * fixtures (tests/test_helper.h:17-22, tolerance 1.0 as in HMM::almost_equal) -- see
 * tests/test_oracle_golden.py -- and by the association analysis in SURVEY.md section 7.
 */
#ifndef SPEC_VITERBI_ORACLE_H
#define SPEC_VITERBI_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint64_t n;                /* states_num */
    uint64_t S;                /* emit_num */
    uint64_t nstart;           /* non_zero_start_probs */
    const uint64_t* start_cols;
    const float* start_vals;   /* -log2 */
    const float* emis;         /* S * n, symbol-major */
    uint64_t ntrans;
    const uint64_t* src;       /* trans_rows */
    const uint64_t* dst;       /* trans_cols */
    const float* prob;         /* trans_probs, -log2 */
} ora_hmm;

/* Status codes (0 = ok). */
#define ORA_OK 0
#define ORA_EINVAL (-1)
#define ORA_ERANGE (-2)
#define ORA_ENOMEM (-3)

/* Non-spec Viterbi of one sequence: out[n] final scores.  bp (nullable) receives
 * (len-1) x n predecessor indices for steps 1..len-1 (-1 = row without terms). */
int ora_viterbi(const ora_hmm* h, const uint64_t* seq, uint64_t len, float* out, int32_t* bp);

/* Decode a path from final scores + backpointers (path[len]). */
int ora_traceback(uint64_t n, uint64_t len, const float* final_scores, const int32_t* bp,
                  int32_t* path);

/* Lowest index of the minimum of v[0..n). */
int64_t ora_argmin(uint64_t n, const float* v);

/* Spec (_spec) Viterbi with `level` (<=1 behaves exactly like level 1). */
int ora_viterbi_spec(const ora_hmm* h, uint32_t level, const uint64_t* seq, uint64_t len,
                     float* out);

/* Level-L precomputed products, dense row-major n x n per key, keys in base-S order with the
 * first observed symbol most significant: out[(key * n + j) * n + m].  Size S^L * n * n. */
int ora_spec_products(const ora_hmm* h, uint32_t level, float* out);

/* Spec Viterbi of many sequences sharing one set of level-L products: out[nseq * n]. */
int ora_viterbi_spec_batch(const ora_hmm* h, uint32_t level, uint64_t nseq, const uint64_t* offsets,
                           const uint64_t* symbols, float* out);

/* Batch of sequences (CPU baseline): offsets[nseq+1] into symbols; out[nseq * n].
 * nthreads <= 0 means "all available". Returns threads actually used via *used (nullable). */
int ora_viterbi_batch(const ora_hmm* h, uint64_t nseq, const uint64_t* offsets,
                      const uint64_t* symbols, float* out, int nthreads, int* used);

#ifdef __cplusplus
}
#endif

#endif
