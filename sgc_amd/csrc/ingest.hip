// ingest.hip -- torch sparse COO/CSR (int64 indices) -> int32 CSR on gfx950.
//
// The reference hands torch.spmm (utils.py:95) the COO tensor built by
// sparse_mx_to_torch_sparse_tensor (utils.py:23-30): int64 [2, nnz] indices,
// fp32 values, in scipy's .tocoo() order, is_coalesced() == False.  torch's
// CPU kernel applies the entries of each row in STORAGE order and never
// merges duplicates.  A CSR that keeps every entry and,
// inside each row, the storage order -- a stable sort by row -- therefore
// feeds the SpMM the same FMA chain.
//
// Fast path (the reference's own S is lexsorted): one streaming pass checks
// ranges and sortedness and narrows col/val into place; a second pass writes
// row_ptr from the row transitions.  Unsorted input: stable LSD radix sort
// (the library's own, sort.hip) of (row, position) pairs, then a gather.
#include "common.h"
#include "sort.h"

namespace sgc {

enum : uint32_t { kRowsSorted = 1u, kColsAscending = 2u, kOutOfRange = 4u };

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n) {
    int64_t b = (n + kBlock - 1) / kBlock;
    return (int)std::max<int64_t>(1, std::min<int64_t>(b, 8192));
}

// flags word starts at kRowsSorted|kColsAscending; bits are cleared/set here.
__global__ void check_narrow_kernel(const int64_t *__restrict__ rows, const int64_t *__restrict__ cols,
                                    const float *__restrict__ vals, int64_t nnz, int64_t n_rows,
                                    int64_t n_cols, int32_t *__restrict__ col_idx,
                                    float *__restrict__ val_out, uint32_t *__restrict__ flags) {
    uint32_t clear = 0, set = 0;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnz;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = rows[k], c = cols[k];
        if (r < 0 || r >= n_rows || c < 0 || c >= n_cols) set |= kOutOfRange;
        if (k + 1 < nnz) {
            const int64_t r2 = rows[k + 1];
            if (r > r2) clear |= kRowsSorted | kColsAscending;
            else if (r == r2 && c >= cols[k + 1]) clear |= kColsAscending;
        }
        col_idx[k] = (int32_t)c;
        val_out[k] = vals[k];
    }
    // at most one atomic per thread (the grid-stride loop folded its bits)
    if (clear) atomicAnd(flags, ~clear);
    if (set) atomicOr(flags, set);
}

// row_ptr[i] = first k with rows[k] >= i, for row-sorted rows (any int type).
template <typename IdxT>
__global__ void row_ptr_from_sorted_kernel(const IdxT *__restrict__ rows, int64_t nnz,
                                           int64_t n_rows, int32_t *__restrict__ row_ptr) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k <= nnz;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t lo = (k == 0) ? -1 : (int64_t)rows[k - 1];
        const int64_t hi = (k == nnz) ? n_rows : (int64_t)rows[k];
        for (int64_t i = lo + 1; i <= hi; ++i) row_ptr[i] = (int32_t)k;
    }
}

__global__ void narrow_rows_iota_kernel(const int64_t *__restrict__ rows, int64_t nnz,
                                        uint32_t *__restrict__ keys, int32_t *__restrict__ pos) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnz;
         k += (int64_t)gridDim.x * blockDim.x) {
        keys[k] = (uint32_t)rows[k];
        pos[k] = (int32_t)k;
    }
}

__global__ void gather_kernel(const int32_t *__restrict__ perm, const int64_t *__restrict__ cols,
                              const float *__restrict__ vals, int64_t nnz,
                              int32_t *__restrict__ col_idx, float *__restrict__ val_out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnz;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t p = perm[k];
        col_idx[k] = (int32_t)cols[p];
        val_out[k] = vals[p];
    }
}

// kColsAscending over an int32 CSR.
__global__ void csr_cols_ascending_kernel(const int32_t *__restrict__ row_ptr,
                                          const int32_t *__restrict__ col_idx, int64_t n_rows,
                                          uint32_t *__restrict__ flags) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_rows;
         i += (int64_t)gridDim.x * blockDim.x) {
        for (int32_t k = row_ptr[i] + 1; k < row_ptr[i + 1]; ++k)
            if (col_idx[k - 1] >= col_idx[k]) {
                atomicAnd(flags, ~kColsAscending);
                break;
            }
    }
}

__global__ void csr64_narrow_kernel(const int64_t *__restrict__ crow, const int64_t *__restrict__ col,
                                    const float *__restrict__ vals, int64_t nnz, int64_t n_rows,
                                    int64_t n_cols, int32_t *__restrict__ row_ptr,
                                    int32_t *__restrict__ col_idx, float *__restrict__ val_out,
                                    uint32_t *__restrict__ flags) {
    const int64_t total = nnz > n_rows + 1 ? nnz : n_rows + 1;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        if (k <= n_rows) {
            const int64_t p = crow[k];
            if (p < 0 || p > nnz || (k > 0 && crow[k - 1] > p)) atomicOr(flags, kOutOfRange);
            row_ptr[k] = (int32_t)p;
        }
        if (k < nnz) {
            const int64_t c = col[k];
            if (c < 0 || c >= n_cols) atomicOr(flags, kOutOfRange);
            col_idx[k] = (int32_t)c;
            val_out[k] = vals[k];
        }
    }
}

struct Carve {
    char *p;
    size_t used = 0;
    template <typename T>
    T *take(size_t n) {
        used = (used + 255) & ~size_t(255);
        T *r = reinterpret_cast<T *>(p ? p + used : nullptr);
        used += n * sizeof(T);
        return r;
    }
};

size_t workspace_layout(int64_t n_rows, int64_t nnz, char *base, uint32_t **flags,
                        uint32_t **keys_in, uint32_t **keys_out, int32_t **pos_in,
                        int32_t **pos_out, void **temp, size_t *temp_bytes) {
    (void)n_rows;
    Carve cv{base};
    *flags = cv.take<uint32_t>(1);
    *keys_in = cv.take<uint32_t>(nnz);
    *keys_out = cv.take<uint32_t>(nnz);
    *pos_in = cv.take<int32_t>(nnz);
    *pos_out = cv.take<int32_t>(nnz);
    *temp_bytes = (size_t)radix_sort_workspace(nnz);
    *temp = cv.take<char>(*temp_bytes);
    return cv.used + 256;
}

}  // namespace

int coo_to_csr_workspace(int64_t n_rows, int64_t nnz, size_t *bytes) {
    SGC_REQUIRE(bytes, SGC_EINVAL, "coo_to_csr_workspace: null");
    SGC_REQUIRE(n_rows >= 0 && nnz >= 0 && n_rows < INT32_MAX && nnz < INT32_MAX, SGC_ERANGE,
                "coo_to_csr: n_rows/nnz beyond int32 CSR");
    uint32_t *f, *a, *b;
    int32_t *c, *d;
    void *t;
    size_t tb;
    *bytes = workspace_layout(n_rows, nnz, nullptr, &f, &a, &b, &c, &d, &t, &tb);
    return SGC_OK;
}

int coo_to_csr(const int64_t *rows, const int64_t *cols, const float *vals, int64_t nnz,
               int64_t n_rows, int64_t n_cols, int32_t *row_ptr, int32_t *col_idx,
               float *val_out, void *ws, size_t ws_bytes, uint32_t *status_host,
               hipStream_t stream) {
    SGC_REQUIRE(n_rows >= 0 && nnz >= 0 && n_cols >= 0, SGC_EINVAL, "coo_to_csr: negative size");
    SGC_REQUIRE(n_rows < INT32_MAX && n_cols < INT32_MAX && nnz < INT32_MAX, SGC_ERANGE,
                "coo_to_csr: n_rows/n_cols/nnz beyond int32 CSR");
    SGC_REQUIRE(row_ptr && ws, SGC_EINVAL, "coo_to_csr: null pointer");
    SGC_REQUIRE(nnz == 0 || (rows && cols && vals && col_idx && val_out), SGC_EINVAL,
                "coo_to_csr: null pointer");
    uint32_t *flags, *keys_in, *keys_out;
    int32_t *pos_in, *pos_out;
    void *temp;
    size_t temp_bytes;
    const size_t need = workspace_layout(n_rows, nnz, (char *)ws, &flags, &keys_in, &keys_out,
                                         &pos_in, &pos_out, &temp, &temp_bytes);
    SGC_REQUIRE(ws_bytes >= need, SGC_ENOMEM, "coo_to_csr: workspace %zu < %zu", ws_bytes, need);

    const uint32_t init = kRowsSorted | kColsAscending;
    SGC_HIP_CHECK(hipMemcpyAsync(flags, &init, sizeof(init), hipMemcpyHostToDevice, stream));
    if (nnz > 0) {
        hipLaunchKernelGGL(check_narrow_kernel, dim3(grid_for(nnz)), dim3(kBlock), 0, stream, rows,
                           cols, vals, nnz, n_rows, n_cols, col_idx, val_out, flags);
        SGC_HIP_CHECK(hipGetLastError());
    }
    uint32_t f = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&f, flags, sizeof(f), hipMemcpyDeviceToHost, stream));
    SGC_HIP_CHECK(hipStreamSynchronize(stream));
    if (f & kOutOfRange) {
        if (status_host) *status_host = f;
        set_error("coo_to_csr: index out of range [0,%lld)x[0,%lld)", (long long)n_rows,
                  (long long)n_cols);
        return SGC_ERANGE;
    }
    if (f & kRowsSorted) {
        hipLaunchKernelGGL(row_ptr_from_sorted_kernel<int64_t>, dim3(grid_for(nnz + 1)), dim3(kBlock),
                           0, stream, rows, nnz, n_rows, row_ptr);
        SGC_HIP_CHECK(hipGetLastError());
    } else {
        hipLaunchKernelGGL(narrow_rows_iota_kernel, dim3(grid_for(nnz)), dim3(kBlock), 0, stream,
                           rows, nnz, keys_in, pos_in);
        SGC_HIP_CHECK(hipGetLastError());
        const int rc = radix_sort_pairs(keys_in, pos_in, keys_out, pos_out, nnz,
                                        (uint32_t)std::max<int64_t>(0, n_rows - 1), false, temp,
                                        (int64_t)temp_bytes, stream);
        if (rc != SGC_OK) return rc;
        hipLaunchKernelGGL(gather_kernel, dim3(grid_for(nnz)), dim3(kBlock), 0, stream, pos_out,
                           cols, vals, nnz, col_idx, val_out);
        SGC_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(row_ptr_from_sorted_kernel<uint32_t>, dim3(grid_for(nnz + 1)),
                           dim3(kBlock), 0, stream, keys_out, nnz, n_rows, row_ptr);
        SGC_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(csr_cols_ascending_kernel, dim3(grid_for(n_rows)), dim3(kBlock), 0,
                           stream, row_ptr, col_idx, n_rows, flags);
        SGC_HIP_CHECK(hipGetLastError());
        SGC_HIP_CHECK(hipMemcpyAsync(&f, flags, sizeof(f), hipMemcpyDeviceToHost, stream));
        SGC_HIP_CHECK(hipStreamSynchronize(stream));
    }
    if (status_host) *status_host = f;
    return SGC_OK;
}

int csr64_to_csr(const int64_t *crow, const int64_t *col, const float *vals, int64_t nnz,
                 int64_t n_rows, int64_t n_cols, int32_t *row_ptr, int32_t *col_idx,
                 float *val_out, uint32_t *status_host, hipStream_t stream) {
    SGC_REQUIRE(n_rows >= 0 && nnz >= 0 && n_cols >= 0, SGC_EINVAL, "csr64_to_csr: negative size");
    SGC_REQUIRE(n_rows < INT32_MAX && n_cols < INT32_MAX && nnz < INT32_MAX, SGC_ERANGE,
                "csr64_to_csr: beyond int32 CSR");
    SGC_REQUIRE(crow && row_ptr && (nnz == 0 || (col && vals && col_idx && val_out)), SGC_EINVAL,
                "csr64_to_csr: null pointer");
    uint32_t *flags = nullptr;
    SGC_HIP_CHECK(hipMallocAsync((void **)&flags, sizeof(uint32_t), stream));
    const uint32_t init = kRowsSorted | kColsAscending;
    SGC_HIP_CHECK(hipMemcpyAsync(flags, &init, sizeof(init), hipMemcpyHostToDevice, stream));
    const int64_t total = nnz > n_rows + 1 ? nnz : n_rows + 1;
    hipLaunchKernelGGL(csr64_narrow_kernel, dim3(grid_for(total)), dim3(kBlock), 0, stream, crow,
                       col, vals, nnz, n_rows, n_cols, row_ptr, col_idx, val_out, flags);
    SGC_HIP_CHECK(hipGetLastError());
    uint32_t f = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&f, flags, sizeof(f), hipMemcpyDeviceToHost, stream));
    SGC_HIP_CHECK(hipStreamSynchronize(stream));
    if (!(f & kOutOfRange) && n_rows > 0) {
        hipLaunchKernelGGL(csr_cols_ascending_kernel, dim3(grid_for(n_rows)), dim3(kBlock), 0,
                           stream, row_ptr, col_idx, n_rows, flags);
        SGC_HIP_CHECK(hipGetLastError());
        SGC_HIP_CHECK(hipMemcpyAsync(&f, flags, sizeof(f), hipMemcpyDeviceToHost, stream));
        SGC_HIP_CHECK(hipStreamSynchronize(stream));
    }
    SGC_HIP_CHECK(hipFreeAsync(flags, stream));
    if (status_host) *status_host = f;
    SGC_REQUIRE(!(f & kOutOfRange), SGC_ERANGE, "csr64_to_csr: index out of range");
    return SGC_OK;
}

SGC_WARM_UNIT(warm_ingest)

}  // namespace sgc
