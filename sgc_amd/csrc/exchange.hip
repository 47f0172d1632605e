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
// for i < rows, j < cols.  Grid y = segment; each wave copies whole rows, LPR
// lanes per row (64 / LPR rows per wave-instruction), V floats per lane.
#include <algorithm>

#include "common.h"

namespace sgc {

namespace {

constexpr int kMaxBlockSegs = 64;

struct CopySeg {
    int64_t src_off, dst_off;  // floats
    int32_t rows, cols;
};

struct CopyArgs {
    CopySeg seg[kMaxBlockSegs];
};

template <int V, int LPR>
__global__ __launch_bounds__(256) void copy_blocks_kernel(const float *__restrict__ src,
                                                          int64_t lds, float *__restrict__ dst,
                                                          int64_t ldd, CopyArgs a) {
    using VT = typename Vec<V>::T;
    const CopySeg s = a.seg[blockIdx.y];
    constexpr int R = kWave / LPR;  // rows per wave-instruction
    const int lane = threadIdx.x & (kWave - 1);
    const int sub = lane / LPR, l = lane - sub * LPR;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
    const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    const int cv = s.cols / V;
    for (int64_t r = w0 * R + sub; r < s.rows; r += waves * R) {
        const VT *sr = reinterpret_cast<const VT *>(src + s.src_off + r * lds);
        VT *dr = reinterpret_cast<VT *>(dst + s.dst_off + r * ldd);
        for (int c = l; c < cv; c += LPR) dr[c] = sr[c];
    }
}

template <int V>
hipError_t launch_lpr(int lpr, const float *src, int64_t lds, float *dst, int64_t ldd,
                      const CopyArgs &a, int nseg, int64_t blocks, hipStream_t s) {
    const dim3 grid((unsigned)blocks, (unsigned)nseg);
    switch (lpr) {
        case 8:
            hipLaunchKernelGGL((copy_blocks_kernel<V, 8>), grid, dim3(256), 0, s, src, lds, dst, ldd, a);
            break;
        case 16:
            hipLaunchKernelGGL((copy_blocks_kernel<V, 16>), grid, dim3(256), 0, s, src, lds, dst, ldd, a);
            break;
        case 32:
            hipLaunchKernelGGL((copy_blocks_kernel<V, 32>), grid, dim3(256), 0, s, src, lds, dst, ldd, a);
            break;
        default:
            hipLaunchKernelGGL((copy_blocks_kernel<V, 64>), grid, dim3(256), 0, s, src, lds, dst, ldd, a);
            break;
    }
    return hipGetLastError();
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
    int64_t max_rows = 0, max_cols = 0;
    for (int s = 0; s < nseg; ++s) {
        const int64_t *q = segs + 6 * s;  // src_row, src_col, dst_row, dst_col, rows, cols
        SGC_REQUIRE(q[0] >= 0 && q[1] >= 0 && q[2] >= 0 && q[3] >= 0 && q[4] >= 0 && q[5] >= 0 &&
                        q[4] < INT32_MAX && q[5] < INT32_MAX,
                    SGC_EINVAL, "copy_blocks: bad segment %d", s);
        SGC_REQUIRE(q[5] == 0 || (q[1] + q[5] <= lds && q[3] + q[5] <= ldd), SGC_EINVAL,
                    "copy_blocks: segment %d columns past the row stride", s);
        if (q[4] == 0 || q[5] == 0) continue;
        a.seg[n] = CopySeg{q[0] * lds + q[1], q[2] * ldd + q[3], (int32_t)q[4], (int32_t)q[5]};
        for (int64_t x : {q[1], q[3], q[5]})
            while (V > 1 && x % V) V >>= 1;
        max_rows = std::max(max_rows, q[4]);
        max_cols = std::max(max_cols, q[5]);
        ++n;
    }
    if (n == 0) return SGC_OK;
    while (V > 1 && (lds % V || ldd % V || reinterpret_cast<uintptr_t>(src) % (4 * V) ||
                     reinterpret_cast<uintptr_t>(dst) % (4 * V)))
        V >>= 1;
    int lpr = 8;  // lanes per row: the vectors of the widest segment, up to the wave
    while (lpr < kWave && lpr * V < max_cols) lpr <<= 1;
    const int64_t rows_per_block = 4 * (kWave / lpr);
    const int64_t blocks = std::max<int64_t>(
        1, std::min<int64_t>((max_rows + rows_per_block - 1) / rows_per_block, 4096 / n + 1));
    hipError_t e = V == 4   ? launch_lpr<4>(lpr, src, lds, dst, ldd, a, n, blocks, stream)
                   : V == 2 ? launch_lpr<2>(lpr, src, lds, dst, ldd, a, n, blocks, stream)
                            : launch_lpr<1>(lpr, src, lds, dst, ldd, a, n, blocks, stream);
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "copy_blocks launch failed: %s", hipGetErrorString(e));
    return SGC_OK;
}

SGC_WARM_UNIT(warm_exchange)

}  // namespace sgc
