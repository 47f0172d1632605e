// subgraph.hip -- the induced sub-graph B = A[idx][:, idx] on gfx950
// (the inductive Reddit path).
//
// Reference: load_reddit_data takes train_adj = adj[train_index, :][:, train_index]
// on the un-normalised A + A^T (utils.py:116-117) and normalises it like the
// full graph (utils.py:123-124 -> normalization.py:5-12).  New row i is old row
// idx[i]; an entry (r, c) survives when c is in idx and becomes column
// inv[c], its position in idx.  The result here is CANONICAL CSR (ascending
// unique columns), fp64 values: exactly what the reference's normalisation
// makes of scipy's slice (coo + eye -> csr sums duplicates and sorts), so
// sgc_augnorm_count/fill turn it into the reference's S_train bit for bit.
//
// count: inv[] by atomicCAS over idx (duplicates and out-of-range ids are
//        flagged: a duplicated id would duplicate rows AND columns, which the
//        caller must handle on the host), one wave per new row counts the kept
//        entries, an exclusive scan gives out_row_ptr;
// fill:  one wave per new row compacts its kept entries with a ballot prefix
//        (old column order); when idx is not ascending the new column ids of a
//        row are not either, and a segmented radix sort by column fixes that.
#include "common.h"

#include <hipcub/hipcub.hpp>

namespace sgc {

namespace {

enum : uint32_t { kDuplicate = 1u, kAscending = 2u, kOutOfRange = 4u };

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

inline int grid_for(int64_t items, int per_block) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((items + per_block - 1) / per_block, 16384));
}

inline size_t up256(size_t b) { return (b + 255) & ~size_t(255); }

__global__ void invert_index_kernel(const int64_t *__restrict__ idx, int64_t m, int64_t n,
                                    int32_t *__restrict__ inv, uint32_t *__restrict__ flags) {
    uint32_t clear = 0, set = 0;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < m;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t old = idx[k];
        if (old < 0 || old >= n) {
            set |= kOutOfRange;
            continue;
        }
        if (k + 1 < m && !(old < idx[k + 1])) clear |= kAscending;
        if (atomicCAS(&inv[old], -1, (int32_t)k) != -1) set |= kDuplicate;
    }
    if (clear) atomicAnd(flags, ~clear);
    if (set) atomicOr(flags, set);
}

__global__ __launch_bounds__(kBlock) void sub_count_kernel(const int32_t *__restrict__ row_ptr,
                                                          const int32_t *__restrict__ col,
                                                          const int64_t *__restrict__ idx, int64_t m,
                                                          const int32_t *__restrict__ inv,
                                                          int32_t *__restrict__ counts) {
    const int lane = threadIdx.x & (kWave - 1);
    for (int64_t i = blockIdx.x * (int64_t)kWavesPerBlock + threadIdx.x / kWave; i < m;
         i += (int64_t)gridDim.x * kWavesPerBlock) {
        const int64_t r = idx[i];
        const int32_t k0 = row_ptr[r], k1 = row_ptr[r + 1];
        int c = 0;
        for (int32_t k = k0 + lane; k < k1; k += kWave) c += inv[col[k]] >= 0;
#pragma unroll
        for (int o = kWave / 2; o > 0; o >>= 1) c += __shfl_xor(c, o, kWave);
        if (lane == 0) counts[i] = c;
    }
}

__global__ __launch_bounds__(kBlock) void sub_fill_kernel(
    const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const double *__restrict__ val, const int64_t *__restrict__ idx, int64_t m,
    const int32_t *__restrict__ inv, const int32_t *__restrict__ out_ptr,
    int32_t *__restrict__ out_col, double *__restrict__ out_val) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (kWave - lane));  // lanes < this one
    for (int64_t i = blockIdx.x * (int64_t)kWavesPerBlock + threadIdx.x / kWave; i < m;
         i += (int64_t)gridDim.x * kWavesPerBlock) {
        const int64_t r = idx[i];
        const int32_t k0 = row_ptr[r], k1 = row_ptr[r + 1];
        int32_t base = out_ptr[i];
        for (int32_t kb = k0; kb < k1; kb += kWave) {
            const int32_t k = kb + lane;
            int32_t nc = -1;
            if (k < k1) nc = inv[col[k]];
            const bool keep = nc >= 0;
            const uint64_t mask = __ballot(keep);
            if (keep) {
                const int32_t o = base + __popcll(mask & below);
                out_col[o] = nc;
                out_val[o] = val[k];
            }
            base += __popcll(mask);
        }
    }
}

struct Layout {  // workspace carve-up shared by count and fill
    uint32_t *flags;
    int32_t *inv;
    int32_t *counts;
    char *scan_tmp;
    size_t scan_bytes;
    int32_t *keys_alt;
    double *vals_alt;
    char *sort_tmp;
    size_t sort_bytes;
    size_t total;
};

Layout carve(void *ws, int64_t n, int64_t m, int64_t nnz) {
    Layout L{};
    size_t scan_bytes = 0, sort_bytes = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, (const int32_t *)nullptr,
                                           (int32_t *)nullptr, (int)std::max<int64_t>(m, 1));
    (void)hipcub::DeviceSegmentedRadixSort::SortPairs(
        nullptr, sort_bytes, (const int32_t *)nullptr, (int32_t *)nullptr,
        (const double *)nullptr, (double *)nullptr, (int)std::max<int64_t>(nnz, 1),
        (int)std::max<int64_t>(m, 1), (const int32_t *)nullptr, (const int32_t *)nullptr);
    char *p = (char *)(((uintptr_t)ws + 255) & ~uintptr_t(255));
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char *q = p + off;
        off += up256(bytes);
        return q;
    };
    L.flags = (uint32_t *)take(sizeof(uint32_t));
    L.inv = (int32_t *)take(sizeof(int32_t) * std::max<int64_t>(n, 1));
    L.counts = (int32_t *)take(sizeof(int32_t) * std::max<int64_t>(m, 1));
    L.scan_bytes = scan_bytes + 256;
    L.scan_tmp = take(L.scan_bytes);
    L.keys_alt = (int32_t *)take(sizeof(int32_t) * std::max<int64_t>(nnz, 1));
    L.vals_alt = (double *)take(sizeof(double) * std::max<int64_t>(nnz, 1));
    L.sort_bytes = sort_bytes + 256;
    L.sort_tmp = take(L.sort_bytes);
    L.total = off + 256;
    return L;
}

}  // namespace

int64_t subgraph_workspace(int64_t n, int64_t m, int64_t nnz) {
    if (n < 0 || m < 0 || nnz < 0) return -1;
    return (int64_t)carve(nullptr, n, m, nnz).total;
}

int subgraph_count(const int32_t *row_ptr, const int32_t *col, int64_t n, const int64_t *idx,
                   int64_t m, int64_t nnz, int32_t *out_row_ptr, void *ws, int64_t ws_bytes,
                   int64_t *out_nnz_host, uint32_t *status_host, hipStream_t s) {
    SGC_REQUIRE(n >= 0 && n < INT32_MAX && m >= 0 && m < INT32_MAX && nnz >= 0 && nnz < INT32_MAX,
                SGC_ERANGE, "subgraph: sizes beyond int32 CSR");
    SGC_REQUIRE(row_ptr && out_row_ptr && ws && out_nnz_host && (m == 0 || idx) &&
                    (nnz == 0 || col),
                SGC_EINVAL, "subgraph_count: null pointer");
    const Layout L = carve(ws, n, m, nnz);
    SGC_REQUIRE((int64_t)L.total <= ws_bytes, SGC_ENOMEM, "subgraph: workspace %lld < %lld bytes",
                (long long)ws_bytes, (long long)L.total);
    const uint32_t init = kAscending;
    SGC_HIP_CHECK(hipMemcpyAsync(L.flags, &init, sizeof(init), hipMemcpyHostToDevice, s));
    if (n > 0) SGC_HIP_CHECK(hipMemsetAsync(L.inv, 0xFF, sizeof(int32_t) * n, s));
    if (m > 0) {
        hipLaunchKernelGGL(invert_index_kernel, dim3(grid_for(m, kBlock)), dim3(kBlock), 0, s, idx,
                           m, n, L.inv, L.flags);
        SGC_HIP_CHECK(hipGetLastError());
    }
    uint32_t f = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&f, L.flags, sizeof(f), hipMemcpyDeviceToHost, s));
    SGC_HIP_CHECK(hipStreamSynchronize(s));
    if (status_host) *status_host = f;
    SGC_REQUIRE(!(f & kOutOfRange), SGC_ERANGE, "subgraph: an index lies outside [0, %lld)",
                (long long)n);
    SGC_REQUIRE(!(f & kDuplicate), SGC_EINVAL,
                "subgraph: repeated indices (duplicate rows and columns) are not supported");
    SGC_HIP_CHECK(hipMemsetAsync(out_row_ptr, 0, sizeof(int32_t), s));
    if (m > 0) {
        hipLaunchKernelGGL(sub_count_kernel, dim3(grid_for(m, kWavesPerBlock)), dim3(kBlock), 0, s,
                           row_ptr, col, idx, m, L.inv, L.counts);
        SGC_HIP_CHECK(hipGetLastError());
        size_t tb = L.scan_bytes;
        SGC_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(L.scan_tmp, tb, L.counts, out_row_ptr + 1,
                                                       (int)m, s));
    }
    int32_t total = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&total, out_row_ptr + m, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    SGC_HIP_CHECK(hipStreamSynchronize(s));
    *out_nnz_host = total;
    return SGC_OK;
}

int subgraph_fill(const int32_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                  const int64_t *idx, int64_t m, int64_t nnz, const int32_t *out_row_ptr,
                  int32_t *out_col, double *out_val, void *ws, int64_t ws_bytes, hipStream_t s) {
    SGC_REQUIRE(row_ptr && out_row_ptr && ws && (m == 0 || idx), SGC_EINVAL,
                "subgraph_fill: null pointer");
    const Layout L = carve(ws, n, m, nnz);
    SGC_REQUIRE((int64_t)L.total <= ws_bytes, SGC_ENOMEM, "subgraph: workspace too small");
    if (m == 0) return SGC_OK;
    uint32_t f = 0;
    int32_t total = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&f, L.flags, sizeof(f), hipMemcpyDeviceToHost, s));
    SGC_HIP_CHECK(hipMemcpyAsync(&total, out_row_ptr + m, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    SGC_HIP_CHECK(hipStreamSynchronize(s));
    SGC_REQUIRE(!(f & (kDuplicate | kOutOfRange)), SGC_EINVAL,
                "subgraph_fill: run sgc_subgraph_count successfully first");
    SGC_REQUIRE(total <= nnz, SGC_ERANGE, "subgraph_fill: %d entries > nnz(A)", total);
    if (total == 0) return SGC_OK;
    SGC_REQUIRE(out_col && out_val && col && val, SGC_EINVAL, "subgraph_fill: null pointer");
    const bool ascending = f & kAscending;
    int32_t *fc = ascending ? out_col : L.keys_alt;
    double *fv = ascending ? out_val : L.vals_alt;
    hipLaunchKernelGGL(sub_fill_kernel, dim3(grid_for(m, kWavesPerBlock)), dim3(kBlock), 0, s,
                       row_ptr, col, val, idx, m, L.inv, out_row_ptr, fc, fv);
    SGC_HIP_CHECK(hipGetLastError());
    if (!ascending) {
        int bits = 1;
        while ((int64_t(1) << bits) < m) ++bits;
        size_t tb = L.sort_bytes;
        SGC_HIP_CHECK(hipcub::DeviceSegmentedRadixSort::SortPairs(
            L.sort_tmp, tb, L.keys_alt, out_col, L.vals_alt, out_val, (int)total, (int)m,
            out_row_ptr, out_row_ptr + 1, 0, bits, s));
    }
    return SGC_OK;
}

SGC_WARM_UNIT(warm_subgraph)

}  // namespace sgc
