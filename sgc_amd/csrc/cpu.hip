// cpu.hip -- host (CPU) twin of the propagation engine, for CPU tensors.
//
// The reference runs its hot path on the CPU whenever CUDA is off
// (args.py:39 --no-cuda -> citation.py -> utils.py:92-97 with cuda=False), so
// the drop-in must too.  This is product code, not the test oracle: the same
// numerical contract as the HIP kernels --
//     Y[i, f]: acc = +0.0f; for k in row i (CSR order): acc = fmaf(val[k], X[col[k], f], acc)
// (with SGC_SPMM_ACCUMULATE the chain starts from Y[i, f] instead: a later
// column-block pass of the same rows, include/sgc_amd.h)
// -- which is bit-identical to torch.spmm's CPU COO kernel.  Threads own whole
// rows (never a split (row, feature) sum); within a row the feature loop
// vectorises across independent chains (vfmadd, one chain per SIMD lane), so
// the FMA order per element is unchanged.
//
// Host-only code: nothing in this file runs on the GPU.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "common.h"

#if !defined(__HIP_DEVICE_COMPILE__)

namespace sgc {
namespace {

constexpr int64_t kRowsPerTask = 64;

// One output row: y[0:F) = sum over the row's nonzeros, sequential fmaf per element.
__attribute__((always_inline)) inline void row_fma(const int32_t *__restrict__ col,
                                                   const float *__restrict__ val, int64_t k0,
                                                   int64_t k1, const float *__restrict__ X,
                                                   int64_t ldx, float *__restrict__ y, int64_t F,
                                                   bool accum) {
    if (!accum)
        for (int64_t f = 0; f < F; ++f) y[f] = 0.0f;
    for (int64_t k = k0; k < k1; ++k) {
        const float v = val[k];
        const float *__restrict__ xr = X + (int64_t)col[k] * ldx;
        for (int64_t f = 0; f < F; ++f) y[f] = __builtin_fmaf(v, xr[f], y[f]);
    }
}

using RowFn = void (*)(const int32_t *, const float *, int64_t, int64_t, const float *, int64_t,
                       float *, int64_t, bool);

__attribute__((target("avx512f,avx512vl,fma"))) void row_avx512(
    const int32_t *col, const float *val, int64_t k0, int64_t k1, const float *X, int64_t ldx,
    float *y, int64_t F, bool accum) {
    row_fma(col, val, k0, k1, X, ldx, y, F, accum);
}

__attribute__((target("avx2,fma"))) void row_avx2(const int32_t *col, const float *val,
                                                  int64_t k0, int64_t k1, const float *X,
                                                  int64_t ldx, float *y, int64_t F, bool accum) {
    row_fma(col, val, k0, k1, X, ldx, y, F, accum);
}

// No hardware FMA: fmaf from libm (correctly rounded, so still bit-exact).
void row_generic(const int32_t *col, const float *val, int64_t k0, int64_t k1, const float *X,
                 int64_t ldx, float *y, int64_t F, bool accum) {
    if (!accum)
        for (int64_t f = 0; f < F; ++f) y[f] = 0.0f;
    for (int64_t k = k0; k < k1; ++k) {
        const float v = val[k];
        const float *xr = X + (int64_t)col[k] * ldx;
        for (int64_t f = 0; f < F; ++f) y[f] = std::fmaf(v, xr[f], y[f]);
    }
}

RowFn pick_row_fn() {
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
        __builtin_cpu_supports("fma"))
        return row_avx512;
    if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return row_avx2;
    return row_generic;
}

int resolve_threads(int32_t n_threads, int64_t work_items) {
    int t = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    t = std::max(1, t);
    const int64_t cap = std::max<int64_t>(1, work_items);
    return (int)std::min<int64_t>(t, cap);
}

// Run body(task) for task in [0, n_tasks) on `threads` threads (dynamic
// scheduling through one atomic counter: hub rows do not stall a thread's
// fixed share).
template <typename Body>
void parallel_tasks(int64_t n_tasks, int threads, Body body) {
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
        for (;;) {
            const int64_t t = next.fetch_add(1, std::memory_order_relaxed);
            if (t >= n_tasks) return;
            body(t);
        }
    };
    if (threads <= 1) {
        worker();
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(threads - 1);
    for (int i = 0; i < threads - 1; ++i) pool.emplace_back(worker);
    worker();
    for (auto &th : pool) th.join();
}

}  // namespace

int coo_to_csr_cpu(const int64_t *rows, const int64_t *cols, const float *vals, int64_t nnz,
                   int64_t n_rows, int64_t n_cols, int32_t *row_ptr, int32_t *col_idx,
                   float *val_out, uint32_t *status_host) {
    SGC_REQUIRE(n_rows >= 0 && nnz >= 0 && n_cols >= 0, SGC_EINVAL, "coo_to_csr_cpu: negative size");
    SGC_REQUIRE(n_rows < INT32_MAX && n_cols < INT32_MAX && nnz < INT32_MAX, SGC_ERANGE,
                "coo_to_csr_cpu: sizes exceed the int32 CSR limits");
    SGC_REQUIRE(row_ptr && (nnz == 0 || (rows && cols && vals && col_idx && val_out)), SGC_EINVAL,
                "coo_to_csr_cpu: null pointer");
    // Stable counting sort by row: every entry kept, each row in storage
    // order -- the order torch's CPU kernel applies the FMAs in.
    std::vector<int64_t> count((size_t)n_rows + 1, 0);
    bool sorted = true, bad = false;
    for (int64_t k = 0; k < nnz; ++k) {
        const int64_t r = rows[k], c = cols[k];
        if (r < 0 || r >= n_rows || c < 0 || c >= n_cols) {
            bad = true;
            break;
        }
        if (k && r < rows[k - 1]) sorted = false;
        ++count[(size_t)r + 1];
    }
    if (bad) {
        if (status_host) *status_host = 4u | (sorted ? 1u : 0u);
        SGC_REQUIRE(false, SGC_ERANGE, "coo_to_csr_cpu: index out of range");
    }
    for (int64_t i = 0; i < n_rows; ++i) count[(size_t)i + 1] += count[(size_t)i];
    for (int64_t i = 0; i <= n_rows; ++i) row_ptr[i] = (int32_t)count[(size_t)i];
    for (int64_t k = 0; k < nnz; ++k) {
        const int64_t p = count[(size_t)rows[k]]++;
        col_idx[p] = (int32_t)cols[k];
        val_out[p] = vals[k];
    }
    bool ascending = true;
    for (int64_t i = 0; i < n_rows && ascending; ++i)
        for (int32_t k = row_ptr[i] + 1; k < row_ptr[i + 1]; ++k)
            if (col_idx[k] <= col_idx[k - 1]) {
                ascending = false;
                break;
            }
    if (status_host) *status_host = (sorted ? 1u : 0u) | (ascending ? 2u : 0u);
    return SGC_OK;
}

int spmm_cpu(const int32_t *row_ptr, const int32_t *col_idx, const float *val, int64_t row_begin,
             int64_t row_end, const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
             int32_t n_threads, bool accum) {
    SGC_REQUIRE(row_ptr && X && Y, SGC_EINVAL, "spmm_cpu: null pointer");
    SGC_REQUIRE(row_begin >= 0 && row_end >= row_begin && row_end < INT32_MAX, SGC_ERANGE,
                "spmm_cpu: bad row range [%lld, %lld)", (long long)row_begin, (long long)row_end);
    // col_idx / val may be NULL only when the rows hold no nonzeros (an empty shard)
    SGC_REQUIRE((col_idx && val) || row_ptr[row_end] == row_ptr[row_begin], SGC_EINVAL,
                "spmm_cpu: null col_idx/val");
    SGC_REQUIRE(F >= 0 && ldx >= F && ldy >= F, SGC_EINVAL, "spmm_cpu: bad shape");
    const int64_t n = row_end - row_begin;
    if (n == 0 || F == 0) return SGC_OK;
    static const RowFn row = pick_row_fn();
    const int64_t tasks = (n + kRowsPerTask - 1) / kRowsPerTask;
    parallel_tasks(tasks, resolve_threads(n_threads, tasks), [&](int64_t t) {
        const int64_t r0 = row_begin + t * kRowsPerTask;
        const int64_t r1 = std::min(row_end, r0 + kRowsPerTask);
        for (int64_t r = r0; r < r1; ++r)
            row(col_idx, val, row_ptr[r], row_ptr[r + 1], X, ldx, Y + (r - row_begin) * ldy, F,
                accum);
    });
    return SGC_OK;
}

int64_t propagate_cpu_workspace(int64_t n_rows, int64_t F, int32_t K) {
    if (n_rows <= 0 || F <= 0 || K <= 1) return 0;
    return (K >= 3 ? 2 : 1) * n_rows * F * 4;
}

int propagate_cpu(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                  int64_t n_rows, const float *X0, int64_t ldx, float *out, int64_t ldo, int64_t F,
                  int32_t K, void *workspace, int64_t workspace_bytes, int32_t n_threads) {
    SGC_REQUIRE(K >= 0, SGC_EINVAL, "propagate_cpu: negative degree %d", K);
    SGC_REQUIRE(X0 && out && F >= 0 && n_rows >= 0 && ldx >= F && ldo >= F, SGC_EINVAL,
                "propagate_cpu: bad arguments");
    if (K == 0) {
        for (int64_t i = 0; i < n_rows; ++i) std::memcpy(out + i * ldo, X0 + i * ldx, F * 4);
        return SGC_OK;
    }
    if (n_rows == 0 || F == 0) return SGC_OK;
    const int64_t need = propagate_cpu_workspace(n_rows, F, K);
    SGC_REQUIRE(workspace_bytes >= need && (need == 0 || workspace), SGC_ENOMEM,
                "propagate_cpu: workspace %lld < %lld bytes", (long long)workspace_bytes,
                (long long)need);
    float *bufs[2] = {static_cast<float *>(workspace),
                      static_cast<float *>(workspace) + (K >= 3 ? n_rows * F : 0)};
    const float *src = X0;
    int64_t lds = ldx;
    for (int h = 0; h < K; ++h) {
        const bool last = h == K - 1;
        float *dst = last ? out : bufs[h & 1];
        const int64_t ldd = last ? ldo : F;
        const int rc = spmm_cpu(row_ptr, col_idx, val, 0, n_rows, src, lds, dst, ldd, F, n_threads,
                                 false);
        if (rc) return rc;
        src = dst;
        lds = ldd;
    }
    return SGC_OK;
}

}  // namespace sgc

#endif  // !__HIP_DEVICE_COMPILE__
