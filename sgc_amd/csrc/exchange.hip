// exchange.hip -- the data movement around the multi-GPU exchanges
// (sgc_amd.distributed): one launch copies a list of 2-D
// blocks between two row-major fp32 buffers.
//
// The replicated output of the partitioned sgc_precompute (every rank gets
// the whole X_K, as reference utils.py:92-97 returns it) arrives from RCCL as
// all_gather_into_tensor's [P x rows, ld] image -- rank q's column block of a
// row chunk at rows [q*rows, (q+1)*rows) -- and must land in X_K's columns
// [c_q, c_{q+1}); the line partition's tail arrives as [P x B, ld] row
// blocks.  One launch per chunk moves every rank's block (P launches of a
// strided copy each paid a ramp, ~0.05 ms apiece at Reddit shape).
//
// Segment s: dst[dst_row + i, dst_col + j] = src[src_row + i, src_col + j]
// for i < rows, j < cols.  Grid y = segment.  A segment is copied as one flat
// run of rows x cols/V vectors of V floats: lane t of the grid takes vectors
// t, t + T, ..., t + (U-1) T (T = the grid's threads), all U loads issued
// before the stores, so a wave-instruction always covers 64 consecutive
// vectors -- whole rows of a narrow block and the next rows after them --
// instead of one row per instruction with the lanes past the block's width
// idle (a 76-float block on 8-B lanes used 38 of 64 lanes: the round-5
// unpack ran at 3.1 TB/s).
#include <algorithm>

#include "common.h"

namespace sgc {

namespace {

constexpr int kMaxBlockSegs = 64;
constexpr int kCopyU = 4;  // vectors per lane in flight

struct CopySeg {
    int64_t src_off, dst_off;  // floats
    int32_t rows, cols;
};

struct CopyArgs {
    CopySeg seg[kMaxBlockSegs];
};

template <int V>
__global__ __launch_bounds__(256) void copy_blocks_kernel(const float *__restrict__ src,
                                                          int64_t lds, float *__restrict__ dst,
                                                          int64_t ldd, CopyArgs a) {
    using VT = typename Vec<V>::T;
    const CopySeg s = a.seg[blockIdx.y];
    const uint32_t cv = (uint32_t)s.cols / V;  // vectors per row
    const uint32_t total = (uint32_t)s.rows * cv;
    const uint32_t T = gridDim.x * blockDim.x;
    const float *sb = src + s.src_off;
    float *db = dst + s.dst_off;
    for (uint32_t base = blockIdx.x * blockDim.x + threadIdx.x; base < total; base += kCopyU * T) {
        VT v[kCopyU];
        int64_t doff[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const uint32_t idx = base + u * T;
            doff[u] = -1;
            if (idx < total) {
                const uint32_t r = idx / cv, c = idx - r * cv;
                v[u] = *reinterpret_cast<const VT *>(sb + r * lds + (int64_t)c * V);
                doff[u] = r * ldd + (int64_t)c * V;
            }
        }
#pragma unroll
        for (int u = 0; u < kCopyU; ++u)
            if (doff[u] >= 0) *reinterpret_cast<VT *>(db + doff[u]) = v[u];
    }
}

}  // namespace

int launch_copy_blocks(const float *src, int64_t lds, float *dst, int64_t ldd, int32_t nseg,
                       const int64_t *segs, hipStream_t stream) {
    SGC_REQUIRE(nseg >= 0 && nseg <= kMaxBlockSegs, SGC_EINVAL,
                "copy_blocks: %d segments (at most %d)", (int)nseg, kMaxBlockSegs);
    SGC_REQUIRE(nseg == 0 || (src && dst && segs), SGC_EINVAL, "copy_blocks: null pointer");
    SGC_REQUIRE(lds >= 0 && ldd >= 0, SGC_EINVAL, "copy_blocks: negative stride");
    CopyArgs a{};
    int n = 0, V = 4;
    int64_t max_elems = 0;
    for (int s = 0; s < nseg; ++s) {
        const int64_t *q = segs + 6 * s;  // src_row, src_col, dst_row, dst_col, rows, cols
        SGC_REQUIRE(q[0] >= 0 && q[1] >= 0 && q[2] >= 0 && q[3] >= 0 && q[4] >= 0 && q[5] >= 0 &&
                        q[4] < INT32_MAX && q[5] < INT32_MAX,
                    SGC_EINVAL, "copy_blocks: bad segment %d", s);
        SGC_REQUIRE(q[5] == 0 || (q[1] + q[5] <= lds && q[3] + q[5] <= ldd), SGC_EINVAL,
                    "copy_blocks: segment %d columns past the row stride", s);
        if (q[4] == 0 || q[5] == 0) continue;
        // the flat index runs in 32 bits
        SGC_REQUIRE(q[4] * q[5] < (int64_t)1 << 31, SGC_EINVAL,
                    "copy_blocks: segment %d has %lld elements (at most 2^31 - 1)", s,
                    (long long)(q[4] * q[5]));
        a.seg[n] = CopySeg{q[0] * lds + q[1], q[2] * ldd + q[3], (int32_t)q[4], (int32_t)q[5]};
        for (int64_t x : {q[1], q[3], q[5]})
            while (V > 1 && x % V) V >>= 1;
        max_elems = std::max(max_elems, q[4] * q[5]);
        ++n;
    }
    if (n == 0) return SGC_OK;
    while (V > 1 && (lds % V || ldd % V || reinterpret_cast<uintptr_t>(src) % (4 * V) ||
                     reinterpret_cast<uintptr_t>(dst) % (4 * V)))
        V >>= 1;
    // enough workgroups that each lane copies ~kCopyU vectors of the largest
    // segment, at most ~8k in all (a grid-stride loop covers the rest)
    const int64_t per_block = 256LL * kCopyU * V;
    const int64_t blocks = std::max<int64_t>(
        1, std::min<int64_t>((max_elems + per_block - 1) / per_block, 8192 / n + 1));
    const dim3 grid((unsigned)blocks, (unsigned)n);
    if (V == 4)
        hipLaunchKernelGGL((copy_blocks_kernel<4>), grid, dim3(256), 0, stream, src, lds, dst, ldd, a);
    else if (V == 2)
        hipLaunchKernelGGL((copy_blocks_kernel<2>), grid, dim3(256), 0, stream, src, lds, dst, ldd, a);
    else
        hipLaunchKernelGGL((copy_blocks_kernel<1>), grid, dim3(256), 0, stream, src, lds, dst, ldd, a);
    const hipError_t e = hipGetLastError();
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "copy_blocks launch failed: %s", hipGetErrorString(e));
    return SGC_OK;
}

SGC_WARM_UNIT(warm_exchange)

}  // namespace sgc
