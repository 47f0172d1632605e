// spmm.hip -- CSR SpMM  Y = S[rows] . X  for gfx950 (MI355X), bit-exact with
// the reference CPU path (torch.spmm at /root/reference/utils.py:95).
//
// Numerical contract (pinned by tests/golden): every output
// element is ONE sequential fp32 FMA chain over its row's nonzeros in CSR
// order, starting from +0.0f.  So a lane owns features and walks the row's
// nonzeros in order; no (row, feature) sum is ever split across lanes, waves
// or launches.
//
// Mapping (one wavefront = 64 lanes per work item):
//   * light item = one whole row: lane l owns the V-float vectors at
//     features (chunk0 + c)*64V + l*V, c in [0, C): C*V accumulators/lane.
//     Y row reads of X are 64V-float coalesced segments of one X row.
//   * heavy item = one (row, chunk) pair of a row with > heavy_threshold
//     nonzeros: the row is split into its chunks_total feature chunks so a
//     power-law hub runs on chunks_total waves at once (still one FMA chain
//     per element).  Heavy items come first in the grid, sorted by degree
//     (sgc_plan_build), so hubs start at t=0 and overlap the light rows.
//   * (col, val) of 64 consecutive nonzeros are read with one coalesced
//     256-B load each, then broadcast per nonzero with v_readlane into SGPRs:
//     the X row base address is scalar, each lane adds its fixed byte offset
//     (global_load_dwordx{1,2,4} saddr + voffset).
//   * U nonzeros are in flight per wave before their FMAs (U*C*V registers);
//     TLP (up to 8 waves/SIMD) hides the rest of the HBM/MALL latency.
//
// Work items beyond F (ragged last chunk) load a valid address (feature 0)
// and are never stored, so no exec-mask branches sit in the inner loop.
#include "common.h"

#include <algorithm>
#include <vector>

namespace sgc {

// Accumulate the C chunks [chunk0, chunk0 + C) of one row and store them.
template <int V, int C, int U>
__device__ __forceinline__ void row_chunks(const int *__restrict__ col,
                                           const float *__restrict__ val, int k0, int k1,
                                           const float *__restrict__ X, int64_t ldx,
                                           float *__restrict__ yrow, int F, int chunk0,
                                           int lane) {
    using VT = typename Vec<V>::T;
    uint32_t boff[C];
    bool ok[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int f = (chunk0 + c) * (kWave * V) + lane * V;
        ok[c] = f < F;
        boff[c] = ok[c] ? uint32_t(f) * 4u : 0u;
    }
    VT acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int v = 0; v < V; ++v) set_elem<V>(acc[c], v, 0.0f);

    const char *Xb = reinterpret_cast<const char *>(X);
    const int64_t row_bytes = ldx * 4;

    for (int base = k0; base < k1; base += kWave) {
        const int n = min(kWave, k1 - base);
        int my_col = 0;
        float my_val = 0.0f;
        if (lane < n) {
            my_col = col[base + lane];
            my_val = val[base + lane];
        }
        int j = 0;
        for (; j + U <= n; j += U) {
            VT xv[U][C];
            float vv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int cj = __builtin_amdgcn_readlane(my_col, j + u);
                vv[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_val), j + u));
                const char *xr = Xb + (int64_t)cj * row_bytes;
#pragma unroll
                for (int c = 0; c < C; ++c)
                    xv[u][c] = *reinterpret_cast<const VT *>(xr + boff[c]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int c = 0; c < C; ++c)
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        set_elem<V>(acc[c], v,
                                    __builtin_fmaf(vv[u], lane_elem<V>(xv[u][c], v),
                                                   lane_elem<V>(acc[c], v)));
        }
        for (; j < n; ++j) {
            const int cj = __builtin_amdgcn_readlane(my_col, j);
            const float vj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_val), j));
            const char *xr = Xb + (int64_t)cj * row_bytes;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const VT x = *reinterpret_cast<const VT *>(xr + boff[c]);
#pragma unroll
                for (int v = 0; v < V; ++v)
                    set_elem<V>(acc[c], v,
                                __builtin_fmaf(vj, lane_elem<V>(x, v), lane_elem<V>(acc[c], v)));
            }
        }
    }
    char *Yb = reinterpret_cast<char *>(yrow);
#pragma unroll
    for (int c = 0; c < C; ++c)
        if (ok[c]) *reinterpret_cast<VT *>(Yb + boff[c]) = acc[c];
}

template <int V, int C, int U, int UH>
__global__ __launch_bounds__(256) void spmm_csr_kernel(
    const int *__restrict__ row_ptr, const int *__restrict__ col, const float *__restrict__ val,
    const float *__restrict__ X, int64_t ldx, float *__restrict__ Y, int64_t ldy,
    int row_begin, int n_rows, int F, const int *__restrict__ heavy_rows,
    int n_heavy_items, int chunks_total, int heavy_threshold) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wave = __builtin_amdgcn_readfirstlane(
        (int)(blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave)));
    if (wave < n_heavy_items) {
        // heavy (row, chunk) item: only the first feature slice launches them
        if (blockIdx.y != 0) return;
        const int h = (int)wave / chunks_total;
        const int c = (int)wave - h * chunks_total;
        const int row = heavy_rows[h];
        const int k0 = row_ptr[row], k1 = row_ptr[row + 1];
        row_chunks<V, 1, UH>(col, val, k0, k1, X, ldx, Y + (int64_t)(row - row_begin) * ldy, F,
                             c, lane);
        return;
    }
    const int64_t r = wave - n_heavy_items;
    if (r >= n_rows) return;
    const int row = row_begin + (int)r;
    const int k0 = row_ptr[row], k1 = row_ptr[row + 1];
    if (heavy_rows != nullptr && k1 - k0 > heavy_threshold) return;  // done as heavy items
    row_chunks<V, C, U>(col, val, k0, k1, X, ldx, Y + r * ldy, F, blockIdx.y * C, lane);
}

namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

struct LaunchArgs {
    const int *row_ptr;
    const int *col;
    const float *val;
    const float *X;
    int64_t ldx;
    float *Y;
    int64_t ldy;
    int row_begin, n_rows, F;
    const int *heavy_rows;
    int n_heavy_items, chunks_total, heavy_threshold;
    int slices;
    hipStream_t stream;
};

template <int V, int C>
hipError_t launch_vc(const LaunchArgs &a) {
    constexpr int U = (C * V >= 16) ? 2 : (C * V >= 8) ? 4 : 8;
    constexpr int UH = (V == 4) ? 8 : 16;
    const int64_t waves = (int64_t)a.n_heavy_items + a.n_rows;
    const int64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    dim3 grid((unsigned)blocks, (unsigned)a.slices);
    hipLaunchKernelGGL((spmm_csr_kernel<V, C, U, UH>), grid, dim3(kBlock), 0, a.stream,
                       a.row_ptr, a.col, a.val, a.X, a.ldx, a.Y, a.ldy, a.row_begin, a.n_rows,
                       a.F, a.heavy_rows, a.n_heavy_items, a.chunks_total, a.heavy_threshold);
    return hipGetLastError();
}

template <int V, int C>
hipError_t dispatch_c(int c, const LaunchArgs &a) {
    if constexpr (C == 0) {
        return hipErrorInvalidValue;
    } else {
        if (c == C) return launch_vc<V, C>(a);
        return dispatch_c<V, C - 1>(c, a);
    }
}

// Largest per-lane register vector the strides and base pointers allow.
int pick_vec(int64_t F, int64_t ldx, int64_t ldy, const void *X, const void *Y) {
    for (int V : {4, 2}) {
        if (F % V == 0 && ldx % V == 0 && ldy % V == 0 &&
            reinterpret_cast<uintptr_t>(X) % (4 * V) == 0 &&
            reinterpret_cast<uintptr_t>(Y) % (4 * V) == 0)
            return V;
    }
    return 1;
}

constexpr int max_chunks(int V) { return 16 / V; }  // <= 16 accumulators per lane

}  // namespace

int launch_spmm(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                int64_t row_begin, int64_t row_end, const float *X, int64_t ldx, float *Y,
                int64_t ldy, int64_t F, const int32_t *heavy_rows, int64_t n_heavy,
                int32_t heavy_threshold, hipStream_t stream) {
    SGC_REQUIRE(row_ptr && col_idx && val && X && Y, SGC_EINVAL, "spmm: null pointer");
    SGC_REQUIRE(row_begin >= 0 && row_end >= row_begin && row_end < INT32_MAX, SGC_ERANGE,
                "spmm: bad row range [%lld, %lld)", (long long)row_begin, (long long)row_end);
    SGC_REQUIRE(F > 0 && F < (1 << 24), SGC_EINVAL, "spmm: bad feature count %lld", (long long)F);
    SGC_REQUIRE(ldx >= F && ldy >= F, SGC_EINVAL, "spmm: ldx/ldy (%lld/%lld) < F (%lld)",
                (long long)ldx, (long long)ldy, (long long)F);
    SGC_REQUIRE(n_heavy >= 0 && (n_heavy == 0 || heavy_rows), SGC_EINVAL, "spmm: bad plan");
    const int64_t n_rows = row_end - row_begin;
    if (n_rows == 0) return SGC_OK;

    const int V = pick_vec(F, ldx, ldy, X, Y);
    const int chunks_total = (int)((F + kWave * V - 1) / (kWave * V));
    const int cmax = max_chunks(V);
    const int slices = (chunks_total + cmax - 1) / cmax;
    const int C = (chunks_total + slices - 1) / slices;
    const int64_t n_heavy_items = heavy_rows ? n_heavy * chunks_total : 0;
    SGC_REQUIRE(n_heavy_items + n_rows < (int64_t)INT32_MAX, SGC_ERANGE, "spmm: too many items");

    LaunchArgs a{row_ptr, col_idx, val, X, ldx, Y, ldy, (int)row_begin, (int)n_rows, (int)F,
                 heavy_rows, (int)n_heavy_items, chunks_total, heavy_threshold, slices, stream};
    hipError_t e;
    if (V == 4)
        e = dispatch_c<4, max_chunks(4)>(C, a);
    else if (V == 2)
        e = dispatch_c<2, max_chunks(2)>(C, a);
    else
        e = dispatch_c<1, max_chunks(1)>(C, a);
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "spmm launch failed: %s", hipGetErrorString(e));
    return SGC_OK;
}

// ---------------------------------------------------------------------------
// Plan: list the rows with > threshold nonzeros, heaviest first.
__global__ void heavy_rows_kernel(const int *__restrict__ row_ptr, int row_begin, int n_rows,
                                  int threshold, int *__restrict__ out_pairs,
                                  int *__restrict__ count) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_rows;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int row = row_begin + (int)i;
        const int d = row_ptr[row + 1] - row_ptr[row];
        if (d > threshold) {
            const int pos = atomicAdd(count, 1);
            out_pairs[2 * pos] = d;
            out_pairs[2 * pos + 1] = row;
        }
    }
}

int build_plan(const int32_t *row_ptr, int64_t row_begin, int64_t row_end,
               int32_t threshold, int32_t *plan, int64_t capacity, int64_t *n_heavy_host,
               hipStream_t stream) {
    SGC_REQUIRE(row_ptr && plan && n_heavy_host, SGC_EINVAL, "plan: null pointer");
    const int64_t n_rows = row_end - row_begin;
    SGC_REQUIRE(n_rows >= 0 && row_end < INT32_MAX, SGC_ERANGE, "plan: bad row range");
    SGC_REQUIRE(capacity >= 2 * n_rows + 1, SGC_ENOMEM, "plan: capacity %lld < %lld",
                (long long)capacity, (long long)(2 * n_rows + 1));
    *n_heavy_host = 0;
    if (n_rows == 0) return SGC_OK;
    int *count = plan + 2 * n_rows;  // last word is the counter
    SGC_HIP_CHECK(hipMemsetAsync(count, 0, sizeof(int), stream));
    const int blocks = (int)std::min<int64_t>((n_rows + 255) / 256, 4096);
    hipLaunchKernelGGL(heavy_rows_kernel, dim3(blocks), dim3(256), 0, stream, row_ptr,
                       (int)row_begin, (int)n_rows, threshold, plan, count);
    SGC_HIP_CHECK(hipGetLastError());
    int h = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&h, count, sizeof(int), hipMemcpyDeviceToHost, stream));
    SGC_HIP_CHECK(hipStreamSynchronize(stream));
    if (h > 0) {
        std::vector<int> pairs(2 * (size_t)h);
        SGC_HIP_CHECK(hipMemcpyAsync(pairs.data(), plan, pairs.size() * sizeof(int),
                                     hipMemcpyDeviceToHost, stream));
        SGC_HIP_CHECK(hipStreamSynchronize(stream));
        std::vector<std::pair<int, int>> dr(h);
        for (int i = 0; i < h; ++i) dr[i] = {-pairs[2 * i], pairs[2 * i + 1]};
        std::sort(dr.begin(), dr.end());  // degree desc, then row asc
        std::vector<int> rows(h);
        for (int i = 0; i < h; ++i) rows[i] = dr[i].second;
        SGC_HIP_CHECK(hipMemcpyAsync(plan, rows.data(), h * sizeof(int), hipMemcpyHostToDevice,
                                     stream));
        SGC_HIP_CHECK(hipStreamSynchronize(stream));
    }
    *n_heavy_host = h;
    return SGC_OK;
}

}  // namespace sgc
