// gemm_tile.h -- the X . W^T register tile shared by the classifier kernels
// (linear.hip, xent.hip): v_mfma_f32_16x16x4_f32, a wave owns MT x 16 rows of X
// and NT x 16 classes.  Lane l loads V consecutive k of X row (l & 15) of each
// m-tile and of W row (l & 15) of each class tile; MFMA v consumes component
// v, so one step covers 4V values of k (MFMA v sums k = k0 + g*V + v over the
// lane groups g = l >> 4).  The next step's operands are loaded before this
// step's MFMAs (register double buffer): with only a few waves per SIMD the
// loads' latency would otherwise sit on the critical path.
#pragma once
#include "common.h"

namespace sgc {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int V, int MT, int NT>
__device__ __forceinline__ void xwt_tile(const float *const (&xrow)[MT],
                                         const float *const (&wrow)[NT], int K, int g,
                                         f32x4 (&acc)[MT][NT]) {
    using VT = typename Vec<V>::T;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    // Full steps carry no masks: a select on just-loaded registers would force
    // the compiler to wait for the prefetch right after issuing it.
    auto load = [&](int k0, VT (&xd)[MT], VT (&wd)[NT]) {
        const int k = k0 + g * V;
#pragma unroll
        for (int t = 0; t < MT; ++t) xd[t] = *reinterpret_cast<const VT *>(xrow[t] + k);
#pragma unroll
        for (int n = 0; n < NT; ++n) wd[n] = *reinterpret_cast<const VT *>(wrow[n] + k);
    };
    auto mma = [&](const VT (&xd)[MT], const VT (&wd)[NT]) {
#pragma unroll
        for (int v = 0; v < V; ++v)
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[t][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        lane_elem<V>(xd[t], v), lane_elem<V>(wd[n], v), acc[t][n], 0, 0, 0);
    };
    const int Kmain = K - K % (4 * V);
    VT xa[MT], wb[NT], xn[MT], wn[NT];
    int k0 = 0;
    if (Kmain > 0) load(0, xa, wb);
    // two steps per iteration so the double buffer needs no register copies
    for (; k0 + 8 * V <= Kmain; k0 += 8 * V) {
        load(k0 + 4 * V, xn, wn);
        mma(xa, wb);
        if (k0 + 8 * V < Kmain) load(k0 + 8 * V, xa, wb);
        mma(xn, wn);
    }
    if (k0 < Kmain) {  // one full step left (already loaded)
        mma(xa, wb);
        k0 += 4 * V;
    }
    if (k0 < K) {  // ragged tail: lanes past K contribute zeros
        const int k = k0 + g * V;
        const bool ok = k < K;
        const int kk = ok ? k : 0;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            xa[t] = *reinterpret_cast<const VT *>(xrow[t] + kk);
            if (!ok) xa[t] = VT{};
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            wb[n] = *reinterpret_cast<const VT *>(wrow[n] + kk);
            if (!ok) wb[n] = VT{};
        }
        mma(xa, wb);
    }
}

}  // namespace sgc

namespace sgc {

// LDS-staged block tile for the classifier GEMMs: a 256-thread block owns
// kLdsBM = 128 rows of X and every class (NT x 16); wave w computes rows
// [32w, 32w + 32) (MT = 2).  Per K-chunk of 32 the block stages X [128 x 32]
// (16 consecutive threads read one row's 128 B: coalesced) and W [16NT x 32]
// through registers into LDS; W leaves L2 once per block, X arrives in whole
// 128-B lines.
//
// Schedule (round 4; the round-1 tile measured 158 us at Reddit-train shape,
// 31 % of the HBM roofline, with its waves 53 % issue-stalled and 36 %
// parked on waits: profiles/r04/pmc_cls/): the LDS image is double buffered,
// so a chunk costs ONE barrier -- chunk c+1's global loads are in flight and
// its LDS store follows chunk c's MFMAs into the other buffer -- and a lane
// reads its operands of the whole chunk with ds_read_b128 (k permuted: MFMA
// step kk sums k = 8g + kk over the lane groups g, so lane l's eight k of a
// chunk are contiguous), 10 LDS reads per 48 MFMAs instead of 40.  fp32 MFMA
// sums exactly; the k order differs from torch's (tolerance parity).
constexpr int kLdsBM = 128;
constexpr int kLdsBK = 32;
// row stride 36 floats: 16-B aligned rows for ds_read_b128 / ds_write_b64
constexpr int kLdsPad = kLdsBK + 4;

template <int V, int NT>
struct LdsTile {
    float xs[2][kLdsBM][kLdsPad];
    float ws[2][NT * 16][kLdsPad];
};

template <int V, int NT>
__device__ __forceinline__ void xwt_block_tile(const float *__restrict__ X, int64_t ldx,
                                               const float *__restrict__ W, int M, int K, int C,
                                               int m_blk, LdsTile<V, NT> &sm,
                                               f32x4 (&acc)[2][NT]) {
    using VT = typename Vec<V>::T;
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int PER_ROW = kLdsBK / V;                      // vectors per row per chunk
    constexpr int XV = kLdsBM * PER_ROW / 256;               // X vectors per thread
    constexpr int WV = (NT * 16 * PER_ROW + 255) / 256;      // W vectors per thread
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    VT xr[XV], wr[WV];
    auto load = [&](int k0) {
#pragma unroll
        for (int j = 0; j < XV; ++j) {
            const int q = tid + 256 * j;
            const int row = q / PER_ROW, k = k0 + (q % PER_ROW) * V;
            const int m = m_blk + row;
            const bool ok = m < M && k < K;
            xr[j] = *reinterpret_cast<const VT *>(X + (int64_t)(ok ? m : 0) * ldx + (ok ? k : 0));
            if (!ok) xr[j] = VT{};
        }
#pragma unroll
        for (int j = 0; j < WV; ++j) {
            const int q = tid + 256 * j;
            const int c = q / PER_ROW, k = k0 + (q % PER_ROW) * V;
            const bool ok = q < NT * 16 * PER_ROW && c < C && k < K;
            wr[j] = *reinterpret_cast<const VT *>(W + (int64_t)(ok ? c : 0) * K + (ok ? k : 0));
            if (!ok) wr[j] = VT{};
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int j = 0; j < XV; ++j) {
            const int q = tid + 256 * j;
            const int row = q / PER_ROW, kc = (q % PER_ROW) * V;
            *reinterpret_cast<VT *>(&sm.xs[buf][row][kc]) = xr[j];
        }
#pragma unroll
        for (int j = 0; j < WV; ++j) {
            const int q = tid + 256 * j;
            if (q < NT * 16 * PER_ROW) {
                const int c = q / PER_ROW, kc = (q % PER_ROW) * V;
                *reinterpret_cast<VT *>(&sm.ws[buf][c][kc]) = wr[j];
            }
        }
    };
    const int n_chunks = (K + kLdsBK - 1) / kLdsBK;
    load(0);
    store(0);
    __syncthreads();
    for (int c = 0; c < n_chunks; ++c) {
        const int buf = c & 1;
        if (c + 1 < n_chunks) load((c + 1) * kLdsBK);  // in flight during this chunk
        // this lane's 8 k of the chunk (k = 8g .. 8g+7) for its rows / classes
        f4 a[2][2], b[NT][2];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                a[t][h] = *reinterpret_cast<const f4 *>(&sm.xs[buf][w * 32 + t * 16 + i][8 * g + 4 * h]);
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                b[n][h] = *reinterpret_cast<const f4 *>(&sm.ws[buf][n * 16 + i][8 * g + 4 * h]);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[t][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        a[t][kk >> 2][kk & 3], b[n][kk >> 2][kk & 3], acc[t][n], 0, 0, 0);
        if (c + 1 < n_chunks) store(buf ^ 1);  // the other buffer: read last chunk, barrier since
        __syncthreads();
    }
}

}  // namespace sgc
