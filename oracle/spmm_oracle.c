/*
 * oracle/spmm_oracle.c -- CPU restatement of the reference's propagation arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (sgc_amd/, libsgc_amd.so)
 * links, loads or calls this file; only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker.
 *
 * What it restates
 * ----------------
 * Reference hot path: /root/reference/utils.py:92-97
 *
 *     for i in range(degree):
 *         features = torch.spmm(adj, features)          # utils.py:95
 *
 * `adj` is a torch sparse COO fp32 [N,N] built by utils.py:23-30; `features`
 * is dense fp32 [N,F].  The arithmetic lives in a third-party dependency
 * (PyTorch aten sparse addmm, pinned torch==1.6.0 at requirements.txt:9; this
 * image runs 2.10.0).  Its CPU semantics, verified bit-for-bit against the
 * reference's own sgc_precompute by tests/golden/gen_golden.py, are:
 *
 *     Y[r, f] = +0.0
 *     for each stored nonzero k in storage order with row(k) == r:
 *         Y[r, f] = fmaf(val[k], X[col[k], f], Y[r, f])
 *
 * i.e. one sequential IEEE fused multiply-add chain per output element, in
 * the COO storage order of that row's entries, with no coalescing (duplicate
 * (r,c) entries are separate FMAs).  A stable sort of COO by row keeps that
 * per-row order, so a CSR built by a stable counting sort gives the same
 * chain (oracle_coo_to_csr below).
 *
 * Build: see oracle/Makefile (gcc -O2 -fopenmp -ffp-contract=off).  fmaf()
 * is glibc's, which dispatches to the hardware FMA where the host has one.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_OK 0
#define ORACLE_EINVAL 1
#define ORACLE_ERANGE 2
#define ORACLE_ENOMEM 3

/* Stable COO -> CSR (int32) by a counting sort on the row index.
 * Mirrors the order torch.spmm consumes entries in (storage order within a
 * row).  Returns ORACLE_ERANGE if an index is outside [0, n) or n/nnz do not
 * fit int32. */
int oracle_coo_to_csr(int64_t n_rows, int64_t n_cols, int64_t nnz,
                      const int64_t *rows, const int64_t *cols, const float *vals,
                      int32_t *row_ptr, int32_t *col_idx, float *val_out)
{
    if (n_rows < 0 || nnz < 0) return ORACLE_EINVAL;
    if (n_rows >= INT32_MAX || nnz >= INT32_MAX || n_cols >= INT32_MAX) return ORACLE_ERANGE;
    int64_t *cursor = (int64_t *)calloc((size_t)n_rows + 1, sizeof(int64_t));
    if (!cursor) return ORACLE_ENOMEM;
    for (int64_t k = 0; k < nnz; ++k) {
        int64_t r = rows[k], c = cols[k];
        if (r < 0 || r >= n_rows || c < 0 || c >= n_cols) { free(cursor); return ORACLE_ERANGE; }
        cursor[r + 1]++;
    }
    for (int64_t i = 0; i < n_rows; ++i) cursor[i + 1] += cursor[i];
    for (int64_t i = 0; i <= n_rows; ++i) row_ptr[i] = (int32_t)cursor[i];
    for (int64_t k = 0; k < nnz; ++k) {
        int64_t dst = cursor[rows[k]]++;
        col_idx[dst] = (int32_t)cols[k];
        val_out[dst] = vals[k];
    }
    free(cursor);
    return ORACLE_OK;
}

/* One hop Y = S.X over CSR rows [row_begin, row_end): the sequential-FMA chain
 * above.  Y rows are indexed from row_begin (Y[0] is row row_begin), matching
 * the row-sliced C-ABI of the product kernel. */
int oracle_spmm_csr(int64_t row_begin, int64_t row_end, int64_t F,
                    const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                    const float *X, int64_t ldx, float *Y, int64_t ldy)
{
    if (row_end < row_begin || F < 0 || ldx < F || ldy < F) return ORACLE_EINVAL;
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t r = row_begin; r < row_end; ++r) {
        float *y = Y + (r - row_begin) * ldy;
        for (int64_t f = 0; f < F; ++f) y[f] = 0.0f;
        for (int32_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
            const float v = val[k];
            const float *x = X + (int64_t)col_idx[k] * ldx;
            for (int64_t f = 0; f < F; ++f) y[f] = fmaf(v, x[f], y[f]);
        }
    }
    return ORACLE_OK;
}

/* One hop directly from COO in storage order (no sort at all): the literal
 * restatement of aten's CPU COO worker.  Single-threaded like the reference
 * kernel.  Used to pin oracle_coo_to_csr + oracle_spmm_csr on unsorted /
 * duplicate inputs. */
int oracle_spmm_coo(int64_t n_rows, int64_t nnz, int64_t F,
                    const int64_t *rows, const int64_t *cols, const float *vals,
                    const float *X, int64_t ldx, float *Y, int64_t ldy)
{
    if (n_rows < 0 || nnz < 0 || F < 0 || ldx < F || ldy < F) return ORACLE_EINVAL;
    for (int64_t r = 0; r < n_rows; ++r)
        for (int64_t f = 0; f < F; ++f) Y[r * ldy + f] = 0.0f;
    for (int64_t k = 0; k < nnz; ++k) {
        float *y = Y + rows[k] * ldy;
        const float *x = X + cols[k] * ldx;
        const float v = vals[k];
        for (int64_t f = 0; f < F; ++f) y[f] = fmaf(v, x[f], y[f]);
    }
    return ORACLE_OK;
}

/* K hops: X_K = S^K X_0 (utils.py:94-95).  work is caller-provided scratch of
 * n_rows*F floats; out receives X_K (contiguous, ld = F).  K = 0 copies X_0. */
int oracle_propagate(int64_t n_rows, int64_t F, int32_t K,
                     const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                     const float *X0, float *out, float *work)
{
    if (K < 0) return ORACLE_EINVAL;
    if (K == 0) { memcpy(out, X0, sizeof(float) * (size_t)(n_rows * F)); return ORACLE_OK; }
    /* ping-pong so that the last hop lands in `out` */
    float *bufs[2] = { out, work };
    const float *src = X0;
    for (int32_t h = 0; h < K; ++h) {
        float *dst = bufs[(K - 1 - h) & 1];
        int rc = oracle_spmm_csr(0, n_rows, F, row_ptr, col_idx, val, src, F, dst, F);
        if (rc) return rc;
        src = dst;
    }
    return ORACLE_OK;
}

/* Classifier forward in fp64 accumulation (models.py:17-18 -> nn.Linear):
 * Y[m,c] = sum_k X[m,k] W[c,k] + b[c].  A tolerance reference for the MFMA
 * linear kernel, not a bit-exact one (summation order is implementation
 * defined in both torch and the kernel). */
int oracle_linear_f64acc(int64_t M, int64_t K, int64_t C,
                         const float *X, const float *W, const float *b, float *Y)
{
#pragma omp parallel for schedule(static)
    for (int64_t m = 0; m < M; ++m)
        for (int64_t c = 0; c < C; ++c) {
            double acc = b ? (double)b[c] : 0.0;
            for (int64_t k = 0; k < K; ++k) acc += (double)X[m * K + k] * (double)W[c * K + k];
            Y[m * C + c] = (float)acc;
        }
    return ORACLE_OK;
}
