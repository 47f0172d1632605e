// normalize.hip -- on-device augmented normalisation S = D^-1/2 (A+I) D^-1/2
// (reference normalization.py:5-12, then utils.py:25's fp32 rounding), the
// SURVEY.md 8(f) row 1 "next" item: at Reddit shape the reference's host
// scipy pass costs ~7 s, against a ~13 ms propagation.
//
// Bit-exact contract with the reference (scipy 1.15 semantics, restated):
//   * A is canonical CSR (ascending unique columns per row), fp64 values;
//   * A+I: the diagonal entry becomes a_ii + 1.0 (inserted as 1.0 at its
//     sorted position when absent); a result of exactly 0.0 is dropped, as
//     scipy's csr binop prunes zeros;
//   * rowsum_i = sequential fp64 sum of row i of A+I in column order (scipy's
//     coo matvec in storage order);
//   * d = rowsum ** -0.5 with inf -> 0 is computed on the HOST with numpy, as
//     the reference does (sgc_amd/normalization.py drives these kernels);
//   * s_ij = (d_i * a_ij) * d_j in fp64 (two csr_matmat passes), entries equal
//     to 0.0 dropped (csr_matmat prunes zeros), then rounded once to fp32.
// Pass 1 counts each row's A+I entries and sums it; pass 2 writes S.  A row
// whose S entries include zeros (only when some d is 0) is rare; pass 2
// reports them and a compaction pass (pass 3) removes them, keeping order.
#include "common.h"

#include <hipcub/hipcub.hpp>

namespace sgc {

namespace {

enum : uint32_t { kNotCanonical = 1u };

constexpr int kBlock = 256;

inline int blocks_for(int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, 16384));
}

// One thread per row: rows are short on average; the sequential fp64 sum is
// the reference's order, so it cannot be split anyway.
__global__ void augnorm_count_kernel(const int32_t *__restrict__ row_ptr,
                                     const int32_t *__restrict__ col,
                                     const double *__restrict__ val, int64_t n,
                                     int32_t *__restrict__ counts, double *__restrict__ rowsum,
                                     uint32_t *__restrict__ flags) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t k0 = row_ptr[i], k1 = row_ptr[i + 1];
        double acc = 0.0;
        int32_t cnt = 0;
        bool diag_done = false;
        int32_t prev = -1;
        for (int32_t k = k0; k < k1; ++k) {
            const int32_t j = col[k];
            if (j <= prev) atomicOr(flags, kNotCanonical);
            prev = j;
            double a = val[k];
            if (!diag_done && j > i) {  // the absent diagonal goes before column j
                acc = acc + 1.0;
                ++cnt;
                diag_done = true;
            }
            if (j == i) {
                a = a + 1.0;
                diag_done = true;
            }
            if (a != 0.0) {
                acc = acc + a;
                ++cnt;
            }
        }
        if (!diag_done) {
            acc = acc + 1.0;
            ++cnt;
        }
        counts[i] = cnt;
        rowsum[i] = acc;
    }
}

__global__ void augnorm_fill_kernel(const int32_t *__restrict__ row_ptr,
                                    const int32_t *__restrict__ col,
                                    const double *__restrict__ val, int64_t n,
                                    const double *__restrict__ d,
                                    const int32_t *__restrict__ out_ptr,
                                    int32_t *__restrict__ out_col, float *__restrict__ out_val,
                                    int32_t *__restrict__ zero_rows) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t k0 = row_ptr[i], k1 = row_ptr[i + 1];
        const double di = d[i];
        int32_t o = out_ptr[i];
        bool diag_done = false, any_zero = false;
        auto emit = [&](int32_t j, double a) {
            const double s = (di * a) * d[j];
            any_zero |= (s == 0.0);
            out_col[o] = j;
            out_val[o] = (float)s;
            ++o;
        };
        for (int32_t k = k0; k < k1; ++k) {
            const int32_t j = col[k];
            double a = val[k];
            if (!diag_done && j > i) {
                emit((int32_t)i, 1.0);
                diag_done = true;
            }
            if (j == i) {
                a = a + 1.0;
                diag_done = true;
            }
            if (a != 0.0) emit(j, a);
        }
        if (!diag_done) emit((int32_t)i, 1.0);
        zero_rows[i] = any_zero ? 1 : 0;
    }
}

// Drop the entries of S that are exactly 0 (fp64 product), keeping order.
__global__ void augnorm_zero_count_kernel(const int32_t *__restrict__ ptr,
                                          const float *__restrict__ v64_sign_source,
                                          const int32_t *__restrict__ zero_rows, int64_t n,
                                          int32_t *__restrict__ counts) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int32_t c = 0;
        for (int32_t k = ptr[i]; k < ptr[i + 1]; ++k) c += v64_sign_source[k] != 0.0f || !zero_rows[i];
        counts[i] = c;
    }
}

__global__ void augnorm_compact_kernel(const int32_t *__restrict__ ptr,
                                       const int32_t *__restrict__ col,
                                       const float *__restrict__ val,
                                       const int32_t *__restrict__ zero_rows, int64_t n,
                                       const int32_t *__restrict__ new_ptr,
                                       int32_t *__restrict__ out_col, float *__restrict__ out_val) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int32_t o = new_ptr[i];
        for (int32_t k = ptr[i]; k < ptr[i + 1]; ++k)
            if (val[k] != 0.0f || !zero_rows[i]) {
                out_col[o] = col[k];
                out_val[o] = val[k];
                ++o;
            }
    }
}

// exclusive scan of counts[0..n) into ptr[0..n], ptr[n] = total (host-visible)
int scan_counts(const int32_t *counts, int64_t n, int32_t *ptr, void *tmp, size_t tmp_bytes,
                hipStream_t s, int64_t *total_host) {
    SGC_HIP_CHECK(hipMemsetAsync(ptr, 0, sizeof(int32_t), s));
    size_t tb = tmp_bytes;
    SGC_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(tmp, tb, counts, ptr + 1, (int)n, s));
    int32_t t = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&t, ptr + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    SGC_HIP_CHECK(hipStreamSynchronize(s));
    *total_host = t;
    return SGC_OK;
}

}  // namespace

size_t augnorm_scan_temp_bytes(int64_t n) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, bytes, (const int32_t *)nullptr,
                                           (int32_t *)nullptr, (int)std::max<int64_t>(n, 1));
    return bytes + 256;
}

int augnorm_count(const int32_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                  int64_t nnz, int32_t *out_row_ptr, double *rowsum, void *ws, size_t ws_bytes,
                  int64_t *out_nnz_host, uint32_t *status_host, hipStream_t s) {
    SGC_REQUIRE(n >= 0 && n < INT32_MAX && nnz >= 0 && nnz < INT32_MAX, SGC_ERANGE,
                "augnorm: sizes beyond int32 CSR");
    SGC_REQUIRE(row_ptr && out_row_ptr && rowsum && ws && (nnz == 0 || (col && val)), SGC_EINVAL,
                "augnorm: null pointer");
    // workspace: flags | counts[n] | scan temp
    char *p = (char *)(((uintptr_t)ws + 255) & ~uintptr_t(255));
    uint32_t *flags = (uint32_t *)p;
    int32_t *counts = (int32_t *)(p + 256);
    char *tmp = p + 256 + ((n * 4 + 255) & ~int64_t(255));
    const size_t tmp_bytes = augnorm_scan_temp_bytes(n);
    SGC_REQUIRE((size_t)(tmp + tmp_bytes - (char *)ws) <= ws_bytes, SGC_ENOMEM,
                "augnorm: workspace too small");
    SGC_HIP_CHECK(hipMemsetAsync(flags, 0, sizeof(uint32_t), s));
    if (n > 0) {
        hipLaunchKernelGGL(augnorm_count_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, row_ptr,
                           col, val, n, counts, rowsum, flags);
        SGC_HIP_CHECK(hipGetLastError());
    }
    uint32_t f = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&f, flags, sizeof(f), hipMemcpyDeviceToHost, s));
    int64_t total = 0;
    if (n > 0) {
        const int rc = scan_counts(counts, n, out_row_ptr, tmp, tmp_bytes, s, &total);
        if (rc) return rc;
    } else {
        SGC_HIP_CHECK(hipMemsetAsync(out_row_ptr, 0, sizeof(int32_t), s));
        SGC_HIP_CHECK(hipStreamSynchronize(s));
    }
    if (status_host) *status_host = f;
    *out_nnz_host = total;
    SGC_REQUIRE(!(f & kNotCanonical), SGC_EINVAL,
                "augnorm: A is not canonical CSR (columns must ascend strictly within rows)");
    return SGC_OK;
}

int augnorm_fill(const int32_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                 const double *d, int32_t *out_row_ptr, int32_t *out_col, float *out_val,
                 void *ws, size_t ws_bytes, int64_t *out_nnz_host, hipStream_t s) {
    SGC_REQUIRE(n >= 0 && n < INT32_MAX, SGC_ERANGE, "augnorm: n beyond int32");
    SGC_REQUIRE(row_ptr && d && out_row_ptr && ws, SGC_EINVAL, "augnorm_fill: null pointer");
    if (n == 0) {
        *out_nnz_host = 0;
        return SGC_OK;
    }
    // workspace: zero_rows[n] | counts[n] | scan temp | compacted col/val (nnz_out each)
    char *p = (char *)(((uintptr_t)ws + 255) & ~uintptr_t(255));
    int32_t *zero_rows = (int32_t *)p;
    int32_t *counts = (int32_t *)(p + ((n * 4 + 255) & ~int64_t(255)));
    char *tmp = (char *)counts + ((n * 4 + 255) & ~int64_t(255));
    const size_t tmp_bytes = augnorm_scan_temp_bytes(n);
    SGC_REQUIRE((size_t)(tmp + tmp_bytes - (char *)ws) <= ws_bytes, SGC_ENOMEM,
                "augnorm_fill: workspace too small");
    hipLaunchKernelGGL(augnorm_fill_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, row_ptr, col,
                       val, n, d, out_row_ptr, out_col, out_val, zero_rows);
    SGC_HIP_CHECK(hipGetLastError());
    // any row with a zero product?  (only when some d is 0: rows summing to 0)
    int32_t nz_total = 0;
    {
        size_t tb = tmp_bytes;
        int32_t *sum_out = counts;  // reuse: reduce zero_rows into counts[0]
        SGC_HIP_CHECK(hipcub::DeviceReduce::Sum(tmp, tb, zero_rows, sum_out, (int)n, s));
        SGC_HIP_CHECK(hipMemcpyAsync(&nz_total, sum_out, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        SGC_HIP_CHECK(hipStreamSynchronize(s));
    }
    int32_t total = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&total, out_row_ptr + n, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    SGC_HIP_CHECK(hipStreamSynchronize(s));
    if (nz_total > 0) {
        // compact in place through a scratch copy of (col, val)
        int32_t *col_tmp = nullptr;
        float *val_tmp = nullptr;
        int32_t *ptr_tmp = nullptr;
        SGC_HIP_CHECK(hipMallocAsync((void **)&col_tmp, sizeof(int32_t) * std::max(total, 1), s));
        SGC_HIP_CHECK(hipMallocAsync((void **)&val_tmp, sizeof(float) * std::max(total, 1), s));
        SGC_HIP_CHECK(hipMallocAsync((void **)&ptr_tmp, sizeof(int32_t) * (n + 1), s));
        SGC_HIP_CHECK(hipMemcpyAsync(col_tmp, out_col, sizeof(int32_t) * total,
                                     hipMemcpyDeviceToDevice, s));
        SGC_HIP_CHECK(hipMemcpyAsync(val_tmp, out_val, sizeof(float) * total,
                                     hipMemcpyDeviceToDevice, s));
        SGC_HIP_CHECK(hipMemcpyAsync(ptr_tmp, out_row_ptr, sizeof(int32_t) * (n + 1),
                                     hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(augnorm_zero_count_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s,
                           ptr_tmp, val_tmp, zero_rows, n, counts);
        SGC_HIP_CHECK(hipGetLastError());
        int64_t t64 = 0;
        int rc = scan_counts(counts, n, out_row_ptr, tmp, tmp_bytes, s, &t64);
        if (rc) return rc;
        hipLaunchKernelGGL(augnorm_compact_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s,
                           ptr_tmp, col_tmp, val_tmp, zero_rows, n, out_row_ptr, out_col, out_val);
        SGC_HIP_CHECK(hipGetLastError());
        SGC_HIP_CHECK(hipFreeAsync(col_tmp, s));
        SGC_HIP_CHECK(hipFreeAsync(val_tmp, s));
        SGC_HIP_CHECK(hipFreeAsync(ptr_tmp, s));
        SGC_HIP_CHECK(hipStreamSynchronize(s));
        total = (int32_t)t64;
    }
    *out_nnz_host = total;
    return SGC_OK;
}

// COO expansion for torch: rows64[k] = row of entry k, cols64[k] = col[k].
__global__ void csr_to_coo64_kernel(const int32_t *__restrict__ row_ptr,
                                    const int32_t *__restrict__ col, int64_t n,
                                    int64_t *__restrict__ rows64, int64_t *__restrict__ cols64) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        for (int32_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
            rows64[k] = i;
            cols64[k] = col[k];
        }
}

int csr_to_coo64(const int32_t *row_ptr, const int32_t *col, int64_t n, int64_t *rows64,
                 int64_t *cols64, hipStream_t s) {
    SGC_REQUIRE(row_ptr && rows64 && cols64 && n >= 0, SGC_EINVAL, "csr_to_coo64: bad arguments");
    if (n == 0) return SGC_OK;
    hipLaunchKernelGGL(csr_to_coo64_kernel, dim3(blocks_for(n)), dim3(kBlock), 0, s, row_ptr, col,
                       n, rows64, cols64);
    SGC_HIP_CHECK(hipGetLastError());
    return SGC_OK;
}

SGC_WARM_UNIT(warm_normalize)

}  // namespace sgc
