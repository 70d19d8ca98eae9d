/*
 * viterbi_oracle.c -- CPU restatement of the reference GraphBLAS Viterbi semantics.
 * TEST INFRASTRUCTURE ONLY (see viterbi_oracle.h for the file:line map and pinning).
 *
 * Build: -O2 -ffp-contract=off, no fast-math: every fp32 add is rounded on its own, in the
 * association the reference's two GrB_mxm calls impose.
 */
#include "viterbi_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* CSR of T^T: row = destination state, col = source state (GraphBLAS_impl.cpp:38-45 builds
 * T^T from (I = trans_cols, J = trans_rows)).  Columns ascend inside a row; duplicates of one
 * (row, col) keep the FIRST tuple in input order (GrB_FIRST_FP32). */
typedef struct {
    uint64_t n;
    uint64_t* rowptr; /* n + 1 */
    uint64_t* col;
    float* val;
} ora_csr;

typedef struct {
    uint64_t dst, src, order;
} ora_triple;

static int triple_cmp(const void* a, const void* b) {
    const ora_triple* x = (const ora_triple*)a;
    const ora_triple* y = (const ora_triple*)b;
    if (x->dst != y->dst) return x->dst < y->dst ? -1 : 1;
    if (x->src != y->src) return x->src < y->src ? -1 : 1;
    if (x->order != y->order) return x->order < y->order ? -1 : 1;
    return 0;
}

static void csr_free(ora_csr* c) {
    free(c->rowptr);
    free(c->col);
    free(c->val);
    memset(c, 0, sizeof(*c));
}

static int csr_build(const ora_hmm* h, ora_csr* c) {
    memset(c, 0, sizeof(*c));
    c->n = h->n;
    ora_triple* t = (ora_triple*)malloc((h->ntrans ? h->ntrans : 1) * sizeof(ora_triple));
    c->rowptr = (uint64_t*)calloc(h->n + 1, sizeof(uint64_t));
    c->col = (uint64_t*)malloc((h->ntrans ? h->ntrans : 1) * sizeof(uint64_t));
    c->val = (float*)malloc((h->ntrans ? h->ntrans : 1) * sizeof(float));
    if (!t || !c->rowptr || !c->col || !c->val) {
        free(t);
        csr_free(c);
        return ORA_ENOMEM;
    }
    for (uint64_t e = 0; e < h->ntrans; ++e) {
        if (h->src[e] >= h->n || h->dst[e] >= h->n) {
            free(t);
            csr_free(c);
            return ORA_ERANGE;
        }
        t[e].dst = h->dst[e];
        t[e].src = h->src[e];
        t[e].order = e;
    }
    qsort(t, h->ntrans, sizeof(ora_triple), triple_cmp);
    uint64_t nnz = 0;
    for (uint64_t e = 0; e < h->ntrans; ++e) {
        if (e > 0 && t[e].dst == t[e - 1].dst && t[e].src == t[e - 1].src) continue; /* FIRST */
        c->col[nnz] = t[e].src;
        c->val[nnz] = h->prob[t[e].order];
        c->rowptr[t[e].dst + 1]++;
        ++nnz;
    }
    for (uint64_t j = 0; j < h->n; ++j) c->rowptr[j + 1] += c->rowptr[j];
    free(t);
    return ORA_OK;
}

/* Dense start column, +inf where absent, first duplicate wins (GraphBLAS_impl.cpp:15-21). */
static int start_build(const ora_hmm* h, float* start) {
    unsigned char* seen = (unsigned char*)calloc(h->n ? h->n : 1, 1);
    if (!seen) return ORA_ENOMEM;
    for (uint64_t j = 0; j < h->n; ++j) start[j] = INFINITY;
    for (uint64_t i = 0; i < h->nstart; ++i) {
        uint64_t c = h->start_cols[i];
        if (c >= h->n) {
            free(seen);
            return ORA_ERANGE;
        }
        if (!seen[c]) {
            start[c] = h->start_vals[i];
            seen[c] = 1;
        }
    }
    free(seen);
    return ORA_OK;
}

static int check_seq(const ora_hmm* h, const uint64_t* seq, uint64_t len) {
    if (len == 0) return ORA_EINVAL;
    for (uint64_t i = 0; i < len; ++i)
        if (seq[i] >= h->S) return ORA_ERANGE;
    return ORA_OK;
}

/* diag(E[s0]) (x) start  (GraphBLAS_impl.cpp:59) */
static void first_step(const ora_hmm* h, const float* start, uint64_t s0, float* v) {
    const float* e = h->emis + s0 * h->n;
    for (uint64_t j = 0; j < h->n; ++j) v[j] = e[j] + start[j];
}

/* One observation: v'[j] = min_k fl(fl(E[o][j] + T^T[j][k]) + v[k])  (GraphBLAS_impl.cpp:65-70).
 * bp (nullable): lexicographic argmin over (value, k); rows without terms get -1. */
static void step(const ora_hmm* h, const ora_csr* c, uint64_t o, const float* v, float* out,
                 int32_t* bp) {
    const float* e = h->emis + o * h->n;
    for (uint64_t j = 0; j < h->n; ++j) {
        float best = INFINITY;
        int64_t arg = -1;
        const float ej = e[j];
        for (uint64_t p = c->rowptr[j]; p < c->rowptr[j + 1]; ++p) {
            const float masked = ej + c->val[p];       /* diag(E[o]) (x) T^T */
            const float term = masked + v[c->col[p]];  /* (.) (x) v          */
            if (arg < 0 || term < best) {              /* columns ascend: ties keep lowest k */
                best = term;
                arg = (int64_t)c->col[p];
            }
        }
        out[j] = best;
        if (bp) bp[j] = (int32_t)arg;
    }
}

static int viterbi_with(const ora_hmm* h, const ora_csr* c, const float* start,
                        const uint64_t* seq, uint64_t len, float* out, int32_t* bp) {
    float* a = (float*)malloc(h->n * sizeof(float) + 4);
    float* b = (float*)malloc(h->n * sizeof(float) + 4);
    if (!a || !b) {
        free(a);
        free(b);
        return ORA_ENOMEM;
    }
    first_step(h, start, seq[0], a);
    for (uint64_t i = 1; i < len; ++i) {
        step(h, c, seq[i], a, b, bp ? bp + (i - 1) * h->n : NULL);
        float* t = a;
        a = b;
        b = t;
    }
    memcpy(out, a, h->n * sizeof(float));
    free(a);
    free(b);
    return ORA_OK;
}

int ora_viterbi(const ora_hmm* h, const uint64_t* seq, uint64_t len, float* out, int32_t* bp) {
    if (!h || !seq || !out || h->n == 0) return ORA_EINVAL;
    int rc = check_seq(h, seq, len);
    if (rc) return rc;
    ora_csr c;
    rc = csr_build(h, &c);
    if (rc) return rc;
    float* start = (float*)malloc(h->n * sizeof(float));
    if (!start) {
        csr_free(&c);
        return ORA_ENOMEM;
    }
    rc = start_build(h, start);
    if (!rc) rc = viterbi_with(h, &c, start, seq, len, out, bp);
    free(start);
    csr_free(&c);
    return rc;
}

int64_t ora_argmin(uint64_t n, const float* v) {
    if (n == 0) return -1;
    uint64_t best = 0;
    for (uint64_t j = 1; j < n; ++j)
        if (v[j] < v[best]) best = j;
    return (int64_t)best;
}

int ora_traceback(uint64_t n, uint64_t len, const float* final_scores, const int32_t* bp,
                  int32_t* path) {
    if (len == 0 || n == 0) return ORA_EINVAL;
    int64_t s = ora_argmin(n, final_scores);
    path[len - 1] = (int32_t)s;
    for (uint64_t t = len - 1; t >= 1; --t) {
        s = (s < 0) ? -1 : bp[(t - 1) * n + (uint64_t)s];
        path[t - 1] = (int32_t)s;
    }
    return ORA_OK;
}

int ora_viterbi_batch(const ora_hmm* h, uint64_t nseq, const uint64_t* offsets,
                      const uint64_t* symbols, float* out, int nthreads, int* used) {
    if (!h || !offsets || !out || h->n == 0) return ORA_EINVAL;
    for (uint64_t q = 0; q < nseq; ++q) {
        int rc = check_seq(h, symbols + offsets[q], offsets[q + 1] - offsets[q]);
        if (rc) return rc;
    }
    ora_csr c;
    int rc = csr_build(h, &c);
    if (rc) return rc;
    float* start = (float*)malloc(h->n * sizeof(float));
    if (!start) {
        csr_free(&c);
        return ORA_ENOMEM;
    }
    rc = start_build(h, start);
    int used_threads = 1;
    int fail = rc;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    used_threads = nthreads;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : fail)
    for (int64_t q = 0; q < (int64_t)nseq; ++q) {
        if (rc) continue;
        fail |= viterbi_with(h, &c, start, symbols + offsets[q], offsets[q + 1] - offsets[q],
                             out + (uint64_t)q * h->n, NULL);
    }
#else
    (void)nthreads;
    for (uint64_t q = 0; q < nseq && !rc; ++q)
        fail |= viterbi_with(h, &c, start, symbols + offsets[q], offsets[q + 1] - offsets[q],
                             out + q * h->n, NULL);
#endif
    if (used) *used = used_threads;
    free(start);
    csr_free(&c);
    return fail ? (rc ? rc : ORA_ENOMEM) : ORA_OK;
}

/* ---- _spec path ------------------------------------------------------------------------- */

static uint64_t ipow(uint64_t b, uint32_t e) {
    uint64_t r = 1;
    while (e--) r *= b;
    return r;
}

/* Dense M_o[j][k] = fl(E[o][j] + T^T[j][k]), +inf where T^T has no entry
 * (GraphBLAS_spec_impl.cpp:146-161). */
static void dense_M(const ora_hmm* h, const ora_csr* c, uint64_t o, float* M) {
    const uint64_t n = h->n;
    for (uint64_t x = 0; x < n * n; ++x) M[x] = INFINITY;
    const float* e = h->emis + o * n;
    for (uint64_t j = 0; j < n; ++j)
        for (uint64_t p = c->rowptr[j]; p < c->rowptr[j + 1]; ++p) M[j * n + c->col[p]] = e[j] + c->val[p];
}

/* res = M_i (x) prev, M_i sparse (pattern of T^T): res[j][m] = min_p fl(M_i[j][p] + prev[p][m])
 * (add_level, GraphBLAS_spec_impl.cpp:25). */
static void left_multiply(const ora_hmm* h, const ora_csr* c, uint64_t i, const float* prev,
                          float* res) {
    const uint64_t n = h->n;
    const float* e = h->emis + i * n;
    for (uint64_t j = 0; j < n; ++j) {
        float* r = res + j * n;
        for (uint64_t m = 0; m < n; ++m) r[m] = INFINITY;
        for (uint64_t p = c->rowptr[j]; p < c->rowptr[j + 1]; ++p) {
            const float mij = e[j] + c->val[p];
            const float* pr = prev + c->col[p] * n;
            for (uint64_t m = 0; m < n; ++m) {
                const float t = mij + pr[m];
                if (t < r[m]) r[m] = t;
            }
        }
    }
}

int ora_spec_products(const ora_hmm* h, uint32_t level, float* out) {
    if (!h || !out || h->n == 0 || level == 0) return ORA_EINVAL;
    ora_csr c;
    int rc = csr_build(h, &c);
    if (rc) return rc;
    const uint64_t n = h->n, nn = n * n;
    /* level 1 = M_o; each further level left-multiplies the newest symbol's M. */
    for (uint64_t o = 0; o < h->S; ++o) dense_M(h, &c, o, out + o * nn);
    float* tmp = NULL;
    for (uint32_t L = 2; L <= level; ++L) {
        const uint64_t prev_keys = ipow(h->S, L - 1);
        free(tmp);
        tmp = (float*)malloc(prev_keys * nn * sizeof(float));
        if (!tmp) {
            csr_free(&c);
            return ORA_ENOMEM;
        }
        memcpy(tmp, out, prev_keys * nn * sizeof(float));
        /* keys are independent: OpenMP over them (each product is computed exactly as above) */
#pragma omp parallel for schedule(dynamic, 1) collapse(2)
        for (uint64_t k = 0; k < prev_keys; ++k)
            for (uint64_t i = 0; i < h->S; ++i)
                left_multiply(h, &c, i, tmp + k * nn, out + (k * h->S + i) * nn);
    }
    free(tmp);
    csr_free(&c);
    return ORA_OK;
}

int ora_viterbi_spec(const ora_hmm* h, uint32_t level, const uint64_t* seq, uint64_t len,
                     float* out) {
    if (!h || !seq || !out || h->n == 0) return ORA_EINVAL;
    int rc = check_seq(h, seq, len);
    if (rc) return rc;
    ora_csr c;
    rc = csr_build(h, &c);
    if (rc) return rc;
    const uint64_t n = h->n;
    float* start = (float*)malloc(n * sizeof(float));
    float* a = (float*)malloc(n * sizeof(float));
    float* b = (float*)malloc(n * sizeof(float));
    float* prod = NULL;
    if (!start || !a || !b) {
        rc = ORA_ENOMEM;
        goto done;
    }
    rc = start_build(h, start);
    if (rc) goto done;
    first_step(h, start, seq[0], a); /* dup of emit_pr_x_start_pr[s0], :54 */
    uint64_t i = 1;
    if (level > 1) {
        prod = (float*)malloc(ipow(h->S, level) * n * n * sizeof(float));
        if (!prod) {
            rc = ORA_ENOMEM;
            goto done;
        }
        rc = ora_spec_products(h, level, prod);
        if (rc) goto done;
        while (len - i >= level) { /* :68-80 */
            uint64_t key = 0;
            for (uint32_t q = 0; q < level; ++q, ++i) key = key * h->S + seq[i];
            const float* H = prod + key * n * n;
#pragma omp parallel for schedule(static)
            for (uint64_t j = 0; j < n; ++j) {
                float best = INFINITY;
                for (uint64_t m = 0; m < n; ++m) {
                    const float t = H[j * n + m] + a[m];
                    if (t < best) best = t;
                }
                b[j] = best;
            }
            float* t = a;
            a = b;
            b = t;
        }
    }
    for (; i < len; ++i) { /* tail, :84-89: M_o (x) v == non-spec step */
        step(h, &c, seq[i], a, b, NULL);
        float* t = a;
        a = b;
        b = t;
    }
    memcpy(out, a, n * sizeof(float));
done:
    free(prod);
    free(start);
    free(a);
    free(b);
    csr_free(&c);
    return rc;
}

/* Spec Viterbi of many sequences with one set of products (the same arithmetic as
 * ora_viterbi_spec, GraphBLAS_spec_impl.cpp:50-89, with spec_with's precompute :146-181 done once
 * as the reference's object does): OpenMP over sequences, each chunk product serial. */
int ora_viterbi_spec_batch(const ora_hmm* h, uint32_t level, uint64_t nseq, const uint64_t* offsets,
                           const uint64_t* symbols, float* out) {
    if (!h || !offsets || !out || h->n == 0) return ORA_EINVAL;
    for (uint64_t q = 0; q < nseq; ++q) {
        int rc = check_seq(h, symbols + offsets[q], offsets[q + 1] - offsets[q]);
        if (rc) return rc;
    }
    ora_csr c;
    int rc = csr_build(h, &c);
    if (rc) return rc;
    const uint64_t n = h->n;
    float* start = (float*)malloc(n * sizeof(float));
    float* prod = NULL;
    if (!start) {
        rc = ORA_ENOMEM;
        goto done;
    }
    rc = start_build(h, start);
    if (rc) goto done;
    if (level > 1) {
        prod = (float*)malloc(ipow(h->S, level) * n * n * sizeof(float));
        if (!prod) {
            rc = ORA_ENOMEM;
            goto done;
        }
        rc = ora_spec_products(h, level, prod);
        if (rc) goto done;
    }
    int fail = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(| : fail)
    for (int64_t q = 0; q < (int64_t)nseq; ++q) {
        const uint64_t* seq = symbols + offsets[q];
        const uint64_t len = offsets[q + 1] - offsets[q];
        float* a = (float*)malloc(n * sizeof(float));
        float* b = (float*)malloc(n * sizeof(float));
        if (!a || !b) {
            free(a);
            free(b);
            fail |= 1;
            continue;
        }
        first_step(h, start, seq[0], a);
        uint64_t i = 1;
        if (level > 1) {
            while (len - i >= level) {
                uint64_t key = 0;
                for (uint32_t k = 0; k < level; ++k, ++i) key = key * h->S + seq[i];
                const float* H = prod + key * n * n;
                for (uint64_t j = 0; j < n; ++j) {
                    float best = INFINITY;
                    for (uint64_t m = 0; m < n; ++m) {
                        const float t = H[j * n + m] + a[m];
                        if (t < best) best = t;
                    }
                    b[j] = best;
                }
                float* t = a;
                a = b;
                b = t;
            }
        }
        for (; i < len; ++i) {
            step(h, &c, seq[i], a, b, NULL);
            float* t = a;
            a = b;
            b = t;
        }
        memcpy(out + (uint64_t)q * n, a, n * sizeof(float));
        free(a);
        free(b);
    }
    if (fail) rc = ORA_ENOMEM;
done:
    free(prod);
    free(start);
    csr_free(&c);
    return rc;
}
