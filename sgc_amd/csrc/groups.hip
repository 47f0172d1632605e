// groups.hip -- column groups of S: the rows' nonzeros split at column cuts
// into G CSRs over the same rows (a schedule for the SpMM; results unchanged).
//
// One hop Y = S.X then runs as G launches over all rows, group 0 plain and
// groups 1.. with SGC_SPMM_ACCUMULATE (each row's FMA chain continues from
// the fp32 value the previous group's launch stored).  With every row's
// columns in ascending order, group g's part of a row is one contiguous run
// of its nonzeros and the runs come in group order, so the chain over groups
// 0..G-1 IS the row's chain in CSR order: bit-identical.  What it buys: each
// launch gathers only the X rows of its column group, so the live part of a
// feature slice is 1/G as large and more of it stays in the per-XCD L2s
// (Reddit shape, one hop at 602 floats: 4.30 -> 3.83 ms at G = 2; RMAT shape
// 31.4 -> 29.5 ms at G = 4; profiles/r03/s14/colgroup*.log).
//
// Layout: the G groups' nonzeros are stored group-major in ONE array pair
// (group 0's runs of rows 0..n-1, then group 1's, ...); group g's row_ptr
// holds absolute offsets into it, so (row_ptr_g, col, val) is an ordinary
// CSR the SpMM, the plan and the hub kernel take unchanged.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace sgc {

namespace {

constexpr int kGroupsMax = 8;
constexpr int kThreads = 256;

struct Cuts {
    int32_t c[kGroupsMax + 1];
};

// first k in [lo, hi) with col[k] >= v (columns ascending within the row)
__device__ __forceinline__ int32_t lower_bound(const int32_t *__restrict__ col, int32_t lo,
                                               int32_t hi, int32_t v) {
    while (lo < hi) {
        const int32_t mid = lo + ((hi - lo) >> 1);
        if (col[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// per-row counts of every group (counts[g * n + r]) and per-block totals
__global__ void colsplit_count_kernel(const int32_t *__restrict__ row_ptr,
                                      const int32_t *__restrict__ col, int32_t n, int32_t chunk,
                                      int G, Cuts cuts, int32_t *__restrict__ counts,
                                      int32_t *__restrict__ block_sums) {
    __shared__ int32_t s_sum[kGroupsMax];
    if (threadIdx.x < kGroupsMax) s_sum[threadIdx.x] = 0;
    __syncthreads();
    const int32_t r0 = blockIdx.x * chunk, r1 = min(n, r0 + chunk);
    int32_t mine[kGroupsMax] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int32_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
        const int32_t k0 = row_ptr[r], k1 = row_ptr[r + 1];
        int32_t lo = k0;
        for (int g = 0; g < G; ++g) {
            const int32_t hi = (g + 1 == G) ? k1 : lower_bound(col, lo, k1, cuts.c[g + 1]);
            counts[(int64_t)g * n + r] = hi - lo;
            mine[g] += hi - lo;
            lo = hi;
        }
    }
    for (int g = 0; g < G; ++g)
        if (mine[g]) atomicAdd(&s_sum[g], mine[g]);
    __syncthreads();
    if (threadIdx.x < G) block_sums[threadIdx.x * gridDim.x + blockIdx.x] = s_sum[threadIdx.x];
}

// exclusive scan of the per-block totals of every group, groups laid out one
// after the other (group g's first block starts after all of group g-1)
__global__ void colsplit_scan_blocks_kernel(int32_t *__restrict__ block_sums, int nblk, int G) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int32_t run = 0;
    for (int g = 0; g < G; ++g)
        for (int b = 0; b < nblk; ++b) {
            const int32_t v = block_sums[g * nblk + b];
            block_sums[g * nblk + b] = run;
            run += v;
        }
}

// row_ptr_g[r] = group g's base + exclusive prefix of counts over the rows;
// block b scans its chunk in tiles of kThreads rows
__global__ void colsplit_rowptr_kernel(const int32_t *__restrict__ counts, int32_t n,
                                       int32_t chunk, int G,
                                       const int32_t *__restrict__ block_off,
                                       int32_t *__restrict__ row_ptrs) {
    __shared__ int32_t s[kThreads];
    __shared__ int32_t s_carry;
    const int32_t r0 = blockIdx.x * chunk, r1 = min(n, r0 + chunk);
    for (int g = 0; g < G; ++g) {
        const int32_t *cnt = counts + (int64_t)g * n;
        int32_t *rp = row_ptrs + (int64_t)g * (n + 1);
        if (threadIdx.x == 0) s_carry = block_off[g * gridDim.x + blockIdx.x];
        __syncthreads();
        for (int32_t base = r0; base < r1; base += kThreads) {
            const int32_t r = base + threadIdx.x;
            const int32_t v = r < r1 ? cnt[r] : 0;
            s[threadIdx.x] = v;
            __syncthreads();
            for (int o = 1; o < kThreads; o <<= 1) {  // inclusive Hillis-Steele scan
                const int32_t add = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
                __syncthreads();
                s[threadIdx.x] += add;
                __syncthreads();
            }
            const int32_t carry = s_carry;
            if (r < r1) rp[r] = carry + s[threadIdx.x] - v;
            __syncthreads();
            if (threadIdx.x == kThreads - 1) s_carry = carry + s[kThreads - 1];
            __syncthreads();
        }
        // the row after the last one: group g's end (= the next group's base)
        if (r1 == n && r0 < r1 && threadIdx.x == 0) rp[n] = s_carry;
        __syncthreads();
    }
}

// one wave per row: copy each group's run of the row to its place
__global__ void colsplit_fill_kernel(const int32_t *__restrict__ row_ptr,
                                     const int32_t *__restrict__ col,
                                     const float *__restrict__ val, int32_t n, int G, Cuts cuts,
                                     const int32_t *__restrict__ row_ptrs,
                                     int32_t *__restrict__ col_out, float *__restrict__ val_out) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; r < n;
         r += waves) {
        const int32_t k0 = row_ptr[r], k1 = row_ptr[r + 1];
        int32_t lo = k0;
        for (int g = 0; g < G; ++g) {
            const int32_t hi = (g + 1 == G) ? k1 : lower_bound(col, lo, k1, cuts.c[g + 1]);
            const int32_t dst = row_ptrs[(int64_t)g * (n + 1) + r];
            for (int32_t k = lo + lane; k < hi; k += kWave) {
                col_out[dst + (k - lo)] = col[k];
                val_out[dst + (k - lo)] = val[k];
            }
            lo = hi;
        }
    }
}

constexpr size_t kAlign = 256;
size_t up(size_t b) { return (b + kAlign - 1) / kAlign * kAlign; }

int nblocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 1023) / 1024)); }

}  // namespace

int64_t colsplit_workspace(int64_t n_rows, int32_t groups) {
    if (n_rows <= 0 || groups <= 0) return (int64_t)kAlign;
    return (int64_t)(up((size_t)groups * n_rows * sizeof(int32_t)) +
                     up((size_t)groups * nblocks(n_rows) * sizeof(int32_t)));
}

int colsplit(const int32_t *row_ptr, const int32_t *col_idx, const float *val, int64_t n_rows,
             int64_t n_cols, int32_t groups, const int32_t *cuts_host, int32_t *row_ptrs,
             int32_t *col_out, float *val_out, void *workspace, int64_t workspace_bytes,
             hipStream_t stream) {
    SGC_REQUIRE(groups >= 1 && groups <= kGroupsMax, SGC_EINVAL,
                "colsplit: groups must be 1..%d", kGroupsMax);
    SGC_REQUIRE(n_rows >= 0 && n_rows < INT32_MAX && n_cols >= 0 && n_cols < INT32_MAX,
                SGC_ERANGE, "colsplit: bad shape");
    SGC_REQUIRE(row_ptr && row_ptrs && cuts_host && workspace, SGC_EINVAL,
                "colsplit: null pointer");
    SGC_REQUIRE(cuts_host[0] == 0 && cuts_host[groups] == n_cols, SGC_EINVAL,
                "colsplit: cuts must run from 0 to n_cols");
    Cuts cuts{};
    for (int g = 0; g <= groups; ++g) {
        SGC_REQUIRE(g == 0 || cuts_host[g] >= cuts_host[g - 1], SGC_EINVAL,
                    "colsplit: cuts must not decrease");
        cuts.c[g] = cuts_host[g];
    }
    if (n_rows == 0) {
        for (int g = 0; g < groups; ++g)
            SGC_HIP_CHECK(hipMemsetAsync(row_ptrs + g, 0, sizeof(int32_t), stream));
        return SGC_OK;
    }
    SGC_REQUIRE(workspace_bytes >= colsplit_workspace(n_rows, groups), SGC_ENOMEM,
                "colsplit: workspace %lld < %lld bytes", (long long)workspace_bytes,
                (long long)colsplit_workspace(n_rows, groups));
    SGC_REQUIRE(col_out && val_out, SGC_EINVAL, "colsplit: null output");
    const int32_t n = (int32_t)n_rows;
    const int nblk = nblocks(n_rows);
    const int32_t chunk = (int32_t)((n_rows + nblk - 1) / nblk);
    char *w = static_cast<char *>(workspace);
    int32_t *counts = reinterpret_cast<int32_t *>(w);
    w += up((size_t)groups * n_rows * sizeof(int32_t));
    int32_t *block_sums = reinterpret_cast<int32_t *>(w);
    hipLaunchKernelGGL(colsplit_count_kernel, dim3(nblk), dim3(kThreads), 0, stream, row_ptr,
                       col_idx, n, chunk, (int)groups, cuts, counts, block_sums);
    SGC_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(colsplit_scan_blocks_kernel, dim3(1), dim3(kWave), 0, stream, block_sums,
                       nblk, (int)groups);
    SGC_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(colsplit_rowptr_kernel, dim3(nblk), dim3(kThreads), 0, stream, counts, n,
                       chunk, (int)groups, block_sums, row_ptrs);
    SGC_HIP_CHECK(hipGetLastError());
    const int fill_blocks = (int)std::min<int64_t>((n_rows + 3) / 4, 8192);
    hipLaunchKernelGGL(colsplit_fill_kernel, dim3(fill_blocks), dim3(kThreads), 0, stream, row_ptr,
                       col_idx, val, n, (int)groups, cuts, row_ptrs, col_out, val_out);
    SGC_HIP_CHECK(hipGetLastError());
    return SGC_OK;
}

// Every row's columns strictly ascending?  (the ingest's status bit 2 for a
// CSR the caller built itself; column groups need it).  Synchronous.
__global__ void cols_ascending_kernel(const int32_t *__restrict__ row_ptr,
                                      const int32_t *__restrict__ col, int64_t n,
                                      int32_t *__restrict__ bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        for (int32_t k = row_ptr[i] + 1; k < row_ptr[i + 1]; ++k)
            if (col[k - 1] >= col[k]) {
                atomicOr(bad, 1);
                break;
            }
    }
}

int csr_cols_ascending(const int32_t *row_ptr, const int32_t *col_idx, int64_t n_rows,
                       hipStream_t stream, bool *ascending) {
    SGC_REQUIRE(row_ptr && ascending, SGC_EINVAL, "cols_ascending: null pointer");
    *ascending = true;
    if (n_rows <= 0) return SGC_OK;
    int32_t *bad = nullptr;
    SGC_HIP_CHECK(hipMallocAsync((void **)&bad, sizeof(int32_t), stream));
    SGC_HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(int32_t), stream));
    const int blocks = (int)std::min<int64_t>((n_rows + 255) / 256, 4096);
    hipLaunchKernelGGL(cols_ascending_kernel, dim3(blocks), dim3(256), 0, stream, row_ptr,
                       col_idx, n_rows, bad);
    SGC_HIP_CHECK(hipGetLastError());
    int32_t h = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, stream));
    SGC_HIP_CHECK(hipFreeAsync(bad, stream));
    SGC_HIP_CHECK(hipStreamSynchronize(stream));
    *ascending = h == 0;
    return SGC_OK;
}

// The size rule of sgc_amd/propagate.py column_groups_for (measured,
// DESIGN.md 4.2): G = 1 below 4 M nonzeros, under 128 features or at 129-256
// (the one-row kernel's single slice); 4 from 64 M nonzeros; else 2.
// SGC_AMD_COLUMN_GROUPS=G forces G, as in the Python layer.
int column_groups_rule(int64_t nnz, int64_t width) {
    static const int forced = [] {
        const char *e = getenv("SGC_AMD_COLUMN_GROUPS");
        return e && *e ? atoi(e) : 0;
    }();
    if (nnz <= 0) return 1;
    if (forced > 0) return std::min(forced, kGroupsMax);
    if (width < 128 || nnz < (int64_t(1) << 22)) return 1;
    if (nnz >= (int64_t(1) << 26)) return 4;
    if (width > 128 && width <= 256) return 1;
    return 2;
}

SGC_WARM_UNIT(warm_groups)

}  // namespace sgc
