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
// (consecutive threads read one row's 128 B: coalesced) and W [16NT x 32]
// through registers into LDS; W leaves L2 once per block, X arrives in whole
// 128-B lines.
//
// Round 4.  Loads are buffer loads: one descriptor per block for its X rows
// and one for W, each lane's byte offsets computed once, so a chunk's load
// costs one add (the round-1 tile spent ~180 VALU instructions per chunk and
// wave on 64-bit addresses and bounds selects -- 20.8 M VALU vs 4.3 M MFMA per
// launch at Reddit-train shape, profiles/r04/pmc_cls2.log).  Rows past M and
// classes past C lie outside their descriptor's range and load zeros; the
// k >= K tail of the last chunk is zeroed in registers (both operands: a
// product of a zero and an infinity beyond K would still be NaN).  NB = 2
// double-buffers the LDS image (one barrier per chunk, the next chunk's loads
// in flight under the MFMAs); NB = 1 keeps one image (two barriers per chunk,
// half the LDS: twice the blocks per CU).  A lane reads its operands of the
// whole chunk with ds_read_b128 (k permuted: MFMA step kk sums k = 8g + kk
// over the lane groups g, so lane l's eight k of a chunk are contiguous), 10
// LDS reads per 48 MFMAs.  fp32 MFMA sums exactly; the k order differs from
// torch's (tolerance parity).
constexpr int kLdsBM = 128;
constexpr int kLdsBK = 32;
// row stride 36 floats: 16-B aligned rows for ds_read_b128 / ds_write_b64
constexpr int kLdsPad = kLdsBK + 4;
// Out-of-range byte offset for a buffer load (zeros), far from any row.
constexpr uint32_t kOffOOB = 0x80000000u;

template <int V, int NT, int NB = 2>
struct LdsTile {  // 16-B aligned rows: the operand reads are ds_read_b128
    alignas(16) float xs[NB][kLdsBM][kLdsPad];
    alignas(16) float ws[NB][NT * 16][kLdsPad];
};

template <int V>
__device__ __forceinline__ typename Vec<V>::T buffer_load_vec(__amdgpu_buffer_rsrc_t r,
                                                             uint32_t off) {
    if constexpr (V == 4)
        return __builtin_bit_cast(typename Vec<4>::T,
                                  __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    else if constexpr (V == 2)
        return __builtin_bit_cast(typename Vec<2>::T,
                                  __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
    else
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// Host-side precondition of xwt_block_tile: a block's X rows and all of W
// addressable with 31-bit byte offsets.
inline bool block_tile_fits(int64_t ldx, int64_t K, int64_t C) {
    return ldx < (int64_t(1) << 31) / (4 * kLdsBM) && K * C < (int64_t(1) << 29);
}

template <int V, int NT, int NB>
__device__ __forceinline__ void xwt_block_tile(const float *__restrict__ X, int64_t ldx,
                                               const float *__restrict__ W, int M, int K, int C,
                                               int m_blk, LdsTile<V, NT, NB> &sm,
                                               f32x4 (&acc)[2][NT]) {
    using VT = typename Vec<V>::T;
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int PER_ROW = kLdsBK / V;                      // vectors per row per chunk
    constexpr int XV = kLdsBM * PER_ROW / 256;               // X vectors per thread
    constexpr int WN = NT * 16 * PER_ROW;                    // W vectors per chunk
    constexpr int WV = (WN + 255) / 256;                     // W vectors per thread
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[t][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int rows = min(kLdsBM, M - m_blk);  // >= 1
    // descriptors from block-uniform values; the last row ends at column K
    const auto xd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(X + (int64_t)m_blk * ldx), 0,
        (int)(((int64_t)(rows - 1) * ldx + K) * 4), 0x00020000);
    const auto wd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(W), 0, C * K * 4,
                                                      0x00020000);
    uint32_t xo[XV], wo[WV];
#pragma unroll
    for (int j = 0; j < XV; ++j) {
        const int q = tid + 256 * j, row = q / PER_ROW, kq = (q % PER_ROW) * V;
        xo[j] = row < rows ? (uint32_t)(row * ldx + kq) * 4u : kOffOOB;
    }
#pragma unroll
    for (int j = 0; j < WV; ++j) {
        const int q = tid + 256 * j, c = q / PER_ROW, kq = (q % PER_ROW) * V;
        wo[j] = (q < WN && c < C) ? (uint32_t)(c * K + kq) * 4u : kOffOOB;
    }
    VT xr[XV], wr[WV];
    auto load = [&](int k0) {
        const uint32_t kb = (uint32_t)k0 * 4u;
#pragma unroll
        for (int j = 0; j < XV; ++j) xr[j] = buffer_load_vec<V>(xd, xo[j] + kb);
#pragma unroll
        for (int j = 0; j < WV; ++j) wr[j] = buffer_load_vec<V>(wd, wo[j] + kb);
        if (k0 + kLdsBK > K) {  // the ragged last chunk only (uniform branch)
#pragma unroll
            for (int j = 0; j < XV; ++j) {
                const int kq = k0 + ((tid + 256 * j) % PER_ROW) * V;
#pragma unroll
                for (int e = 0; e < V; ++e)
                    if (kq + e >= K) set_elem<V>(xr[j], e, 0.f);
            }
#pragma unroll
            for (int j = 0; j < WV; ++j) {
                const int kq = k0 + ((tid + 256 * j) % PER_ROW) * V;
#pragma unroll
                for (int e = 0; e < V; ++e)
                    if (kq + e >= K) set_elem<V>(wr[j], e, 0.f);
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int j = 0; j < XV; ++j) {
            const int q = tid + 256 * j;
            *reinterpret_cast<VT *>(&sm.xs[buf][q / PER_ROW][(q % PER_ROW) * V]) = xr[j];
        }
#pragma unroll
        for (int j = 0; j < WV; ++j) {
            const int q = tid + 256 * j;
            if (WN % 256 == 0 || q < WN)
                *reinterpret_cast<VT *>(&sm.ws[buf][q / PER_ROW][(q % PER_ROW) * V]) = wr[j];
        }
    };
    const int n_chunks = (K + kLdsBK - 1) / kLdsBK;
    load(0);
    store(0);
    __syncthreads();
    for (int c = 0; c < n_chunks; ++c) {
        const int buf = NB == 2 ? (c & 1) : 0;
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
        if constexpr (NB == 2) {
            if (c + 1 < n_chunks) store(buf ^ 1);  // the other buffer: read last chunk, barrier since
            __syncthreads();
        } else {
            if (c + 1 < n_chunks) {
                __syncthreads();  // every wave has read this chunk's image
                store(0);
                __syncthreads();
            }
        }
    }
}

}  // namespace sgc
