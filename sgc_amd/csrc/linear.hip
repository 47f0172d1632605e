// linear.hip -- SGC classifier forward  Y = X . W^T + b  (reference
// models.py:17-18: nn.Linear(nfeat, nclass)) on gfx950 fp32 MFMA.
//
// v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf chain per output,
// cdna_hip_programming.md 3) -- lane l holds A[l&15][l>>4], B[l>>4][l&15],
// D[4*(l>>4)+r][l&15].  A = 16 rows of X, B = 16 classes of W^T.
//
// A 256-thread block owns 128 rows and all classes (NT x 16, padded); X and
// W chunks are staged through LDS (gemm_tile.h: xwt_block_tile), so X is read
// once from HBM in whole lines and W once per block from L2.  At the Reddit-train
// shape the fp32 MFMA work (2 x 152,410 x 602 x 48 = 8.8 GFLOP, 56 us at
// 157 TF) and the X read (367 MB, ~60 us) are about even.
#include <map>
#include <mutex>
#include <set>
#include <utility>

#include "gemm_tile.h"
#include "split_bf16.h"

namespace sgc {

template <int V, int NT, int NB>
__global__ __launch_bounds__(256) void linear_kernel(const float *__restrict__ X, int64_t ldx,
                                                     const float *__restrict__ W,
                                                     const float *__restrict__ b,
                                                     float *__restrict__ Y, int64_t ldy, int M,
                                                     int K, int C) {
    __shared__ LdsTile<V, NT, NB> sm;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int m_blk = blockIdx.x * kLdsBM;
    f32x4 acc[2][NT];
    xwt_block_tile<V, NT, NB>(X, ldx, W, M, K, C, m_blk, sm, acc);
    const int m0 = m_blk + w * 32;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int c = n * 16 + i;
        if (c >= C) continue;
        const float bias = b ? b[c] : 0.0f;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + t * 16 + g * 4 + r;
                if (m < M) Y[(int64_t)m * ldy + c] = acc[t][n][r] + bias;
            }
    }
}

// ---------------------------------------------------------------------------
// Streaming form (the default where W fits LDS): W^T lives in LDS for the
// whole launch and every wave streams its own 16-row tiles of X straight from
// HBM into MFMA operand registers -- no X staging through LDS, no barrier
// after the one W load, so no wave ever waits for another.
//
// * Grid: one 1024-thread workgroup per CU (W's image is ~123 KB at 48 x 640),
//   persistent; tile t (rows 16t..16t+15) goes to workgroup t mod grid, whose
//   waves take their next tile from an LDS counter.
// * Per 32-k chunk lane (i, g) loads row i's k0+4g .. +3 and k0+16+4g .. +3
//   (two b128, or four b64 on 8-B aligned rows -- ldx = 602 is), so one load
//   instruction reads 64 contiguous bytes of each of its 16 rows and each
//   row's 128-B line is read once per chunk; the loads run kStreamDepth chunks ahead in a register ring
//   (the wave's chunk stream runs on across tile boundaries, with running
//   (tile, chunk) counters: no divisions), so each SIMD keeps ~4 x 4 x 2 KB of
//   X in flight; a slot is reloaded after the MFMAs that read it (no copies).
// * MFMA step kk of a chunk sums k = k0 + 16(kk >> 2) + 4g + (kk & 3) over g
//   (any k permutation shared by both operands sums the same products; fp32
//   MFMA products are exact), W's operands by ds_read_b128 from an
//   XOR-swizzled image (conflict-free in every b128 lane group).
// Measured before these last three points (profiles/r04/cls_diag*.log): the
// same 0.128 ms as the LDS tile, with the loads alone 0.111 and the MFMAs
// alone 0.108 -- per-chunk divisions, operand copies and 75 % LDS
// bank-conflict cycles, not HBM or the MFMA pipe, set both.
// * Loads go through one buffer descriptor over all of X: rows past M read
//   zeros; the last chunk's k >= K are zeroed in registers (X beyond a row is
//   the next row, and 0 x inf would be NaN).
// MFMA work at 152,410 x 602 x 48 is 56 us at the fp32 peak and the X read
// ~58 us at 6.3 TB/s: both pipes must run together.
constexpr int kStreamDepth = 4;  // chunks in flight per wave
constexpr int kStreamWaves = 16;

// DIAG (diagnostics only, sgc_set_tuning("linear_kernel", 3 / 4)): 1 = the
// loads and stores without the MFMAs (the X stream's own time), 2 = the MFMAs
// on registers without the X loads (the MFMA pipe's own time).
// CK: k per chunk, 32 or 64 (a lane holds CK/4 k of a row per chunk; 64 = half
// the per-chunk bookkeeping per MFMA at the same bytes in flight, two chunks
// deep instead of four).
template <int V, int NT, int DIAG = 0, int CK = 32>
__global__ __launch_bounds__(64 * kStreamWaves) void linear_stream_kernel(
    const float *__restrict__ X, int64_t ldx, const float *__restrict__ W,
    const float *__restrict__ b, float *__restrict__ Y, int64_t ldy, int M, int K, int C,
    int Kp) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    using VT = typename Vec<V>::T;
    constexpr int E = CK / 4;              // k per lane per chunk
    constexpr int NV = E / V;              // vector loads per lane per chunk
    constexpr int NJ = E / 4;              // 16-B granules per lane per chunk
    constexpr int D = CK == 32 ? kStreamDepth : kStreamDepth / 2;  // chunks in flight
    // W^T image [NT*16][S], S = K rounded up to 64 floats; the 16-B granule q
    // of row r sits at granule q ^ (r & 15) of its 64-float window, so every
    // ds_read_b128 lane group (4 x 16 lanes, MI355X_MICROARCH.md LDS table)
    // hits 16 distinct 4-bank groups: lane (i, g) reads granule 8c + 4h + g
    // of row n*16 + i (a plain stride leaves 2-way conflicts in two groups).
    extern __shared__ __attribute__((aligned(16))) float sw[];
    const int S = (K + 63) / 64 * 64;
    // the wave index as a scalar: every tile / chunk counter below derives from
    // it and stays in SGPRs, so the per-chunk control flow is scalar branches
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int i = lane & 15, g = lane >> 4;
    // (eight independent loads in flight per thread: the image is ~30 loads
    // per thread, which one at a time cost several microseconds of latency)
    constexpr int kWU = 8;
    for (int base = threadIdx.x; base < NT * 16 * S; base += kWU * 64 * kStreamWaves) {
        float v[kWU];
#pragma unroll
        for (int u = 0; u < kWU; ++u) {
            const int idx = base + u * 64 * kStreamWaves;
            const int r = idx / S, k = idx - r * S;
            v[u] = (idx < NT * 16 * S && r < C && k < K) ? W[(int64_t)r * K + k] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < kWU; ++u) {
            const int idx = base + u * 64 * kStreamWaves;
            const int r = idx / S, k = idx - r * S;
            if (idx < NT * 16 * S) sw[r * S + (((k >> 2) ^ (r & 15)) << 2) + (k & 3)] = v[u];
        }
    }
    __syncthreads();
    const int n_tiles = (M + 15) >> 4;
    // Tiles are dealt per workgroup (t = block + grid * m, 37-38 per CU at the
    // Reddit-train shape) and its 16 waves take the next m from an LDS counter
    // as they go, so every wave stays busy until the CU's list is done (a fixed
    // deal gave some waves 3 tiles and their SIMD-mates 2: the last third of
    // the launch ran on a quarter of the waves).
    int *next = reinterpret_cast<int *>(sw + NT * 16 * S);
    if (threadIdx.x == 0) *next = 0;
    __syncthreads();
    (void)w;
    auto grab = [&]() -> int {
        int m = 0;
        if (lane == 0) m = atomicAdd(next, 1);
        m = __builtin_amdgcn_readfirstlane(m);
        const int t = (int)blockIdx.x + (int)gridDim.x * m;
        return t < n_tiles ? t : -1;
    };
    const int NC = Kp / CK;  // chunks per tile
    const auto xd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(X), 0, (int)((int64_t)M * ldx * 4), 0x00020000);  // < 2^31
    // loader: chunk lc of tile ltile (-1: the CU's list is done)
    int ltile = grab(), lc = 0;
    auto row_off = [&](int tile) -> uint32_t {
        const int row = tile * 16 + i;
        return (tile >= 0 && row < M) ? (uint32_t)((int64_t)row * ldx * 4) + 16u * g : kOffOOB;
    };
    uint32_t lrow = row_off(ltile);
    VT xr[D][NV];
    int stile[D], sc[D];  // each slot's (tile, chunk); tile -1 = none
    auto load = [&](int slot_) {
        stile[slot_] = ltile;
        sc[slot_] = lc;
        if (ltile < 0) return;
        const uint32_t off = lrow + (uint32_t)lc * (CK * 4u);
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            if constexpr (DIAG == 2)
                xr[slot_][q] = VT{} + (float)(off & 7);
            else  // element e = qV.. of the lane: byte 16g + 4(e & 3) + 64(e >> 2)
                xr[slot_][q] = buffer_load_vec<V>(xd, off + ((q * V * 4) & 15) +
                                                          ((q * V * 4) >> 4) * 64);
        }
        if (++lc == NC) {
            lc = 0;
            ltile = grab();
            lrow = row_off(ltile);
        }
    };
#pragma unroll
    for (int u = 0; u < D; ++u) load(u);
    f32x4 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    // W operands of chunk c (granules 8c + 4h + g of rows n*16 + i, swizzled),
    // read one chunk ahead into the other register set, so the MFMAs never
    // wait for their LDS reads
    f4 bw[2][NT][NJ];
    auto read_w = [&](int c, f4 (&dst)[NT][NJ]) {
        const int q0 = c * E;  // the chunk's first granule... of 16 per 64-float window
        const int wbase = (q0 >> 4) * 64;
#pragma unroll
        for (int h = 0; h < NJ; ++h) {
            const int col = wbase + (((((q0 & 15)) + 4 * h + g) ^ i) << 2);
#pragma unroll
            for (int n = 0; n < NT; ++n)
                dst[n][h] = *reinterpret_cast<const f4 *>(&sw[(n * 16 + i) * S + col]);
        }
    };
    // (at NT = 4, or with 64-k chunks, the second set would spill at the
    // 128-VGPR cap of 16 waves: read in place there)
    constexpr bool kPreW = NT <= 3 && CK == 32;
    if constexpr (kPreW) read_w(sc[0], bw[0]);
    static_assert(D % 2 == 0, "the W register sets alternate per slot");
    for (;;) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const int tile = stile[u], c = sc[u];
            if (tile < 0) return;  // wave-uniform: the stream is in order, so all later slots are empty too
            const int cur = kPreW ? (u & 1) : 0;  // a constant after unrolling
            const int un = (u + 1) % D;
            if constexpr (kPreW) {
                if (stile[un] >= 0) read_w(sc[un], bw[cur ^ 1]);
            } else if constexpr (CK == 32) {
                read_w(c, bw[0]);
            }
            float a[E];
#pragma unroll
            for (int q = 0; q < NV; ++q)
#pragma unroll
                for (int e = 0; e < V; ++e) a[q * V + e] = lane_elem<V>(xr[u][q], e);
            if ((c + 1) * CK > K) {  // the ragged last chunk (uniform)
#pragma unroll
                for (int e = 0; e < E; ++e)
                    if (c * CK + 16 * (e >> 2) + 4 * g + (e & 3) >= K) a[e] = 0.0f;
            }
            if constexpr (DIAG == 1) {
#pragma unroll
                for (int kk = 0; kk < E; ++kk)
                    acc[kk % NT][kk & 3] += a[kk] * bw[cur][0][0][kk & 3];
            } else if constexpr (CK == 32) {
#pragma unroll
                for (int kk = 0; kk < E; ++kk)
#pragma unroll
                    for (int n = 0; n < NT; ++n)
                        acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            a[kk], bw[cur][n][kk >> 2][kk & 3], acc[n], 0, 0, 0);
            } else {  // 64-k chunks: W operands in two halves of two granules (registers)
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    f4 bh[NT][2];
                    const int wbase = c * 64;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int col = wbase + (((4 * (2 * hh + h) + g) ^ i) << 2);
#pragma unroll
                        for (int n = 0; n < NT; ++n)
                            bh[n][h] = *reinterpret_cast<const f4 *>(&sw[(n * 16 + i) * S + col]);
                    }
#pragma unroll
                    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
                        for (int n = 0; n < NT; ++n)
                            acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                a[8 * hh + kk], bh[n][kk >> 2][kk & 3], acc[n], 0, 0, 0);
                }
            }
            // the chunk kStreamDepth ahead into the slot just consumed
            load(u);
            if (c == NC - 1) {  // tile done: D[4g + r][i] = row 4g + r, class n*16 + i
                const int m0 = tile * 16 + 4 * g;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    const int cl = n * 16 + i;
                    if (cl >= C) continue;
                    const float bias = b ? b[cl] : 0.0f;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (m0 + r < M) Y[(int64_t)(m0 + r) * ldy + cl] = acc[n][r] + bias;
                }
#pragma unroll
                for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Split-bf16 streaming form (round 5, the default where its W image fits LDS).
// The fp32 MFMA runs at 1/16 of the bf16 rate, and at the Reddit-train shape
// its 4.34 M MFMAs alone (56 us at peak) are as long as the X stream: the
// round-4 kernel could not overlap the two.  Here every fp32 operand is split
// into three bf16 pieces, x = h + m + l EXACTLY (h = RNE(x), m = RNE(x - h),
// l = x - h - m; each difference is exact by Sterbenz), and x . w is taken as
// the six products that reach fp32 precision -- hh, hm, mh, hl, lh, mm (the
// dropped ml, lm, ll are below 2^-25 of |x||w|) -- on v_mfma_f32_16x16x32_bf16,
// whose bf16 x bf16 products are exact in its fp32 sums: 6/16 of the fp32 MFMA
// time, so the X stream alone sets the pace.  Tolerance parity with fp32
// (test_linear_split_*).  Finite X and W only: an infinite x gives NaN (its
// residual x - h is inf - inf), where torch gives +-inf or NaN; values past
// bf16's largest finite (+-3.39e38) likewise.
// * X stream: per 32-k chunk of a 16-row tile a lane issues two b128 loads,
//   each wave-instruction reading 128 contiguous bytes of each of 8 rows (8
//   lanes per row): instruction 0 rows 0-7, instruction 1 rows 8-15, lane
//   (j, kg) = (l & 15, l >> 4) at byte 16 * (2 kg + (j >> 3)) of the chunk.
//   The round-4 shape (64 B of each of 16 rows, the MFMA operand layout
//   loaded directly) streamed at 2.4-3.2 TB/s, this one at 5.5-5.8
//   (scripts/micro/stream_shape.hip, profiles/r05/stream_shape.log).  One DPP
//   row_ror:8 exchange per register then gives lane (j, kg) floats 8kg..8kg+7
//   of row j -- the bf16 16x16x32 B operand, k in natural order.
// * D = W . X^T (W the A operand): a lane's accumulator holds four
//   consecutive classes of one row, so a tile's output is b128 stores.
// * W's pieces stay in LDS for the whole persistent launch in MFMA-operand
//   order: per 32-k chunk, per class tile, each lane's three 16-B operands
//   side by side (48 B per lane: conflict-free b128 reads, the piece and the
//   tile as immediate offsets, one address add per chunk); the last class
//   tile keeps only its Cl real classes (+ one zero granule for the lanes
//   past them), which is what fits C = 41 at K = 602 (150 KB).  The image is
//   built in-kernel after the first X loads are in flight.
// * The ring of D chunks per wave runs across tiles with compile-time slots
//   (a rolled ring moved registers and selected slots at run time: ~100 extra
//   VALU per chunk).
#ifndef SGC_SPLIT_DEPTH
#define SGC_SPLIT_DEPTH 4
#endif
// chunks in flight per wave (the ring's slots): 4; 6 or 8 stream the loads
// alone 1-2 % faster but the kernel no faster (0.092-0.093 vs 0.090-0.091 ms,
// profiles/r05/linear_ab_depth.log)
constexpr int kSplitDepth = SGC_SPLIT_DEPTH;
#ifndef SGC_SPLIT_HELD
#define SGC_SPLIT_HELD 6
#endif
// Finished tiles a wave holds in registers before it stores them (at NT = 3;
// more at NT <= 2, fewer at NT = 4): stores count in the same vmcnt as the X
// loads, so stores issued while the loads stream make the next chunks'
// counted waits drain the ring.  Held, a wave stores after its last load
// (~4.7 tiles per wave at the Reddit-train shape; a seventh flushes the six).
constexpr int kSplitHeld = SGC_SPLIT_HELD;
template <int U> struct SlotC { static constexpr int value = U; };

// f(SlotC<U>{}) for U = U0 .. D-1 in order, compile-time slots (run_slots
// stops at the first false and returns false).
template <int U, int D, typename F>
__device__ __forceinline__ void each_slot(F &&f) {
    if constexpr (U < D) {
        f(SlotC<U>{});
        each_slot<U + 1, D>(f);
    }
}
template <int U, int D, typename F>
__device__ __forceinline__ bool run_slots(F &&f) {
    if constexpr (U < D) {
        if (!f(SlotC<U>{})) return false;
        return run_slots<U + 1, D>(f);
    } else {
        return true;
    }
}

__device__ __forceinline__ float ror8(float x) {  // lane j of each 16-lane row gets lane j ^ 8's x
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x128, 0xf, 0xf, false));
}

// W image geometry (host and device): bytes per chunk for NT class tiles, the
// last holding Cl classes.
__host__ __device__ constexpr int split_chunk_bytes(int NT, int Cl) {
    return (NT - 1) * 3072 + (4 * Cl + 1) * 48;
}


// DIAG (diagnostics, sgc_set_tuning("linear_kernel", 6 / 7 / 8)): 1 = the
// loads, the exchange and the stores without the split and the MFMAs; 2 = 1
// without the stores; 3 = everything but the stores.
template <int NT, int NW, int DIAG = 0>
__global__ __launch_bounds__(64 * NW) void linear_split_kernel(
    const float *__restrict__ X, int64_t ldx, const float *__restrict__ W,
    const float *__restrict__ b, float *__restrict__ Y, int64_t ldy, int M, int K, int C) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) u32x4 sgr[];
    char *const lds = reinterpret_cast<char *>(sgr);
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, kg = lane >> 4;
    const int NC = (K + 31) / 32;         // chunks per tile
    const int Cl = C - (NT - 1) * 16;     // classes of the last tile, 1..16
    const int cstride = split_chunk_bytes(NT, Cl);
    int *next = reinterpret_cast<int *>(lds + NC * cstride);
    if (threadIdx.x == 0) *next = 0;
    __syncthreads();
    const int n_tiles = (M + 15) >> 4;
    auto grab = [&]() -> int {  // the workgroup's next tile (block + grid * m), or -1
        int m = 0;
        if (lane == 0) m = atomicAdd(next, 1);
        m = __builtin_amdgcn_readfirstlane(m);
        const int t = (int)blockIdx.x + (int)gridDim.x * m;
        return t < n_tiles ? t : -1;
    };
    const auto xd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(X), 0, (int)((int64_t)M * ldx * 4), 0x00020000);  // < 2^31
    const uint32_t seg = 16u * (2 * kg + (j >> 3));
    const uint32_t pitch8 = (uint32_t)(8 * ldx * 4);
    int ltile = grab(), lc = 0;
    uint32_t lrow0 = 0, lrow1 = 0;
    auto rows_of = [&](int tile) {
        const int row = tile * 16 + (j & 7);
        lrow0 = (tile >= 0 && row < M) ? (uint32_t)((int64_t)row * ldx * 4) + seg : kOffOOB;
        lrow1 = (tile >= 0 && row + 8 < M) ? lrow0 + pitch8 : kOffOOB;
    };
    rows_of(ltile);
    constexpr int D = kSplitDepth;
    static_assert(D >= 2 && D <= 8, "ring depth");
    f4 xa[D], xb[D];
    int stile[D], sc[D];
    // Both loads are issued on every path (past the last tile their offsets
    // are out of range: zeros, no memory traffic), so every path has the same
    // loads in flight and the compiler's counted waits stay exact.
    auto load = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        stile[u] = ltile;
        sc[u] = lc;
        const uint32_t co = (uint32_t)lc * 128u;
        xa[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xd, lrow0 + co, 0, 0));
        xb[u] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(xd, lrow1 + co, 0, 0));
        if (ltile >= 0 && ++lc == NC) {
            lc = 0;
            ltile = grab();
            rows_of(ltile);
        }
    };
    // the ring's first chunks are in flight while W's image is built
    each_slot<0, D>(load);
    {
        // one unit = one lane's operand granule of one (chunk, class tile):
        // 8 k of one class, split into its three pieces, stored side by side
        const auto wd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(W), 0,
                                                          (int)((int64_t)C * K * 4), 0x00020000);
        // one unit = 8 k (a granule) of one class row, split into its three
        // pieces and stored at its lane's place in the chunk's operand block;
        // units run along W's rows, so a wave's loads read 2 KB of one row
        // contiguously (in operand order the lanes read 64 different rows:
        // ~10 us of scattered line requests per workgroup)
        const int full = (NT - 1) * 64;
        const int G = NC * 4;  // granules per class row
        constexpr int FU = 8;  // units per thread per round, loads all issued first
        for (int base = threadIdx.x; base < C * G; base += FU * 64 * NW) {
            f4 e[FU][2];
            int dsto[FU];
#pragma unroll
            for (int f = 0; f < FU; ++f) {
                const int idx = base + f * 64 * NW;
                const bool in = idx < C * G;
                const int r = in ? idx / G : 0, g = in ? idx - r * G : 0;
                const int c = g >> 2, kk = g & 3, n = r >> 4, jj = r & 15;
                const int w = n < NT - 1 ? n * 64 + jj + 16 * kk : full + kk * Cl + jj;
                dsto[f] = in ? c * cstride + w * 48 : -1;
                const uint32_t off = (uint32_t)(r * K + 8 * g) * 4u;
                e[f][0] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(wd, off, 0, 0));
                e[f][1] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(wd, off + 16, 0, 0));
                if (8 * g + 8 > K) {  // the row's last granule: k >= K is the next row
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (8 * g + q >= K) e[f][q >> 2][q & 3] = 0.0f;
                }
            }
#pragma unroll
            for (int f = 0; f < FU; ++f) {
                uint32_t h[4], m[4], l[4];
#pragma unroll
                for (int p = 0; p < 4; ++p)
                    split3(e[f][p >> 1][2 * (p & 1)], e[f][p >> 1][2 * (p & 1) + 1], h[p], m[p], l[p]);
                if (dsto[f] >= 0) {
                    char *dst = lds + dsto[f];
                    *reinterpret_cast<u32x4 *>(dst) = u32x4{h[0], h[1], h[2], h[3]};
                    *reinterpret_cast<u32x4 *>(dst + 16) = u32x4{m[0], m[1], m[2], m[3]};
                    *reinterpret_cast<u32x4 *>(dst + 32) = u32x4{l[0], l[1], l[2], l[3]};
                }
            }
        }
        // the zero granule of each chunk's last class tile (its lanes past Cl)
        for (int c = threadIdx.x; c < NC; c += 64 * NW) {
            char *dst = lds + c * cstride + (full + 4 * Cl) * 48;
#pragma unroll
            for (int p = 0; p < 3; ++p) *reinterpret_cast<u32x4 *>(dst + 16 * p) = u32x4{0u, 0u, 0u, 0u};
        }
    }
    __syncthreads();
    // a lane's operand granules: full tile n at bfull + n * 3072, the last
    // tile at blast (the zero granule for lanes past its Cl classes); piece p
    // at + 16 p; chunk c at + c * cstride
    const uint32_t bfull = (uint32_t)lane * 48u;
    const uint32_t blast = (NT - 1) * 3072u + 48u * (uint32_t)(j < Cl ? kg * Cl + j : 4 * Cl);
    // the bias of the lane's classes (n * 16 + 4 kg + r)
    f4 bias[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int cl = n * 16 + 4 * kg + r;
            bias[n][r] = (b && cl < C) ? b[cl] : 0.0f;
        }
    const auto yd = __builtin_amdgcn_make_buffer_rsrc(Y, 0, (int)((int64_t)M * ldy * 4),
                                                      0x00020000);  // < 2^31
    constexpr int PT0 = NT <= 2 ? kSplitHeld + 2 : NT == 3 ? kSplitHeld : kSplitHeld - 2;
    constexpr int PT = PT0 < 1 ? 1 : PT0;
    f4 held[PT][NT];
    uint32_t hrow[PT];
    int nheld = 0;  // uniform
    const int pcl = (NT - 1) * 16 + 4 * kg;  // the lane's last class group
    const bool ppart = pcl + 4 > C;           // partial (or empty): b32 stores
    // Y row offset -> its classes: full groups of four by b128, the partial
    // last group by b32; every store issued, out-of-range offsets when empty
    auto store_tile = [&](const f4 (&o)[NT], uint32_t yrow) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int cl0 = n * 16 + 4 * kg;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o[n]), yd,
                                                   cl0 + 4 <= C ? yrow + 4u * cl0 : kOffOOB, 0, 0);
        }
        // the partial group of four (only one lane group has one: C % 4 classes)
        if (C % 4) {  // uniform
            // (the elements as separate values first: extracting them from
            // the vector the b128 store took was miscompiled -- every b32
            // store wrote element 0)
            const u32x4 pe = __builtin_bit_cast(u32x4, o[NT - 1]);
            const uint32_t e0 = pe.x, e1 = pe.y, e2 = pe.z;
            auto off = [&](int r) { return (ppart && pcl + r < C) ? yrow + 4u * (pcl + r) : kOffOOB; };
            __builtin_amdgcn_raw_buffer_store_b32(e0, yd, off(0), 0, 0);
            if (C % 4 >= 2) __builtin_amdgcn_raw_buffer_store_b32(e1, yd, off(1), 0, 0);
            if (C % 4 == 3) __builtin_amdgcn_raw_buffer_store_b32(e2, yd, off(2), 0, 0);
        }
    };
    auto flush = [&]() {
#pragma unroll
        for (int t = 0; t < PT; ++t)
            if (t < nheld) store_tile(held[t], hrow[t]);  // uniform
        nheld = 0;
    };
    f32x4 accH[NT], accL[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) accH[n] = accL[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    float diag_sum = 0.0f;
    const bool low = j < 8;
    auto step = [&](auto uc) -> bool {  // false: the stream is done (uniform)
        constexpr int u = decltype(uc)::value;
        const int tile = stile[u], c = sc[u];
        if (tile < 0) return false;
        // W operands of chunk c
        u32x4 bw[NT][3];
        {
            const uint32_t coff = (uint32_t)c * (uint32_t)cstride;
            const char *af = lds + bfull + coff;
            const char *al = lds + blast + coff;
#pragma unroll
            for (int n = 0; n < NT; ++n)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    bw[n][p] = *reinterpret_cast<const u32x4 *>(
                        (n < NT - 1 ? af + n * 3072 : al) + 16 * p);
        }
        const f4 A = xa[u], B = xb[u];
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float t = ror8(low ? B[e] : A[e]);
            v[e] = low ? A[e] : t;
            v[4 + e] = low ? t : B[e];
        }
        load(uc);  // the chunk D ahead into the slot just consumed
        if ((c + 1) * 32 > K) {  // the ragged last chunk (uniform)
#pragma unroll
            for (int e = 0; e < 8; ++e)
                if (c * 32 + 8 * kg + e >= K) v[e] = 0.0f;
        }
        if constexpr (DIAG == 1 || DIAG == 2) {
#pragma unroll
            for (int e = 0; e < 8; ++e) accH[0][e & 3] += v[e];
        } else {
            uint32_t ah[4], am[4], al[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) split3(v[2 * p], v[2 * p + 1], ah[p], am[p], al[p]);
            const bf16x8_t Xh = __builtin_bit_cast(bf16x8_t, u32x4{ah[0], ah[1], ah[2], ah[3]});
            const bf16x8_t Xm = __builtin_bit_cast(bf16x8_t, u32x4{am[0], am[1], am[2], am[3]});
            const bf16x8_t Xl = __builtin_bit_cast(bf16x8_t, u32x4{al[0], al[1], al[2], al[3]});
            auto wb = [&](int n, int p) { return __builtin_bit_cast(bf16x8_t, bw[n][p]); };
#pragma unroll
            for (int n = 0; n < NT; ++n)
                accH[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb(n, 0), Xh, accH[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n)
                accL[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb(n, 1), Xh, accL[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n)
                accL[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb(n, 0), Xm, accL[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n)
                accL[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb(n, 2), Xh, accL[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n)
                accL[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb(n, 0), Xl, accL[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n)
                accL[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb(n, 1), Xm, accL[n], 0, 0, 0);
        }
        if (c == NC - 1) {  // tile done: D[4 kg + r][j] = class n * 16 + 4 kg + r, row j
            const int row = tile * 16 + j;  // rows past M: out-of-range offsets, dropped
            const uint32_t yrow = row < M ? (uint32_t)((int64_t)row * ldy * 4) : kOffOOB;
            if constexpr (DIAG >= 2) {  // diagnostics without the stores
#pragma unroll
                for (int n = 0; n < NT; ++n)
#pragma unroll
                    for (int r = 0; r < 4; ++r) diag_sum += accH[n][r] + accL[n][r];
            } else {
                if (nheld == PT) flush();
#pragma unroll
                for (int t = 0; t < PT; ++t)
                    if (t == nheld) {  // uniform
#pragma unroll
                        for (int n = 0; n < NT; ++n) held[t][n] = accH[n] + accL[n] + bias[n];
                        hrow[t] = yrow;
                    }
                ++nheld;
            }
#pragma unroll
            for (int n = 0; n < NT; ++n) accH[n] = accL[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        return true;
    };
    for (;;) {
        if (!run_slots<0, D>(step)) break;
    }
    if constexpr (DIAG >= 2) {
        if (diag_sum == 12345.0f) Y[lane] = diag_sum;  // keeps the work live
    } else {
        flush();
    }
}

// 0 = auto (split-bf16 streaming where W's images fit LDS, else fp32
// streaming where W^T fits and the rows are 8-B aligned, else the LDS tile),
// 1 = the LDS tile, 2 = fp32 streaming (3 / 4: its DIAG forms, wrong results
// by design), 5 = split-bf16 streaming (6: its loads-only DIAG form).
// Set through sgc_set_tuning("linear_kernel").
int g_linear_kernel = 0;
// k per chunk of the streaming kernel, 32 or 64 (64: forward 0.1237-0.1238
// vs 0.1263-0.1273 ms at the Reddit-train shape, profiles/r04/classifier_ck64_ab.log).
// Set through sgc_set_tuning("linear_ck").
int g_linear_ck = 64;

// One LDS image per block (two barriers per chunk, half the LDS: twice the
// blocks per CU) measured faster than the double buffer at the Reddit-train
// shape: forward 0.128-0.130 vs 0.146-0.152 ms (profiles/r04/classifier_v3_*.log).
int g_tile_buffers = 1;

namespace {

template <int V, int NT>
hipError_t launch_linear(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                         int64_t ldy, int M, int K, int C, hipStream_t s) {
    const int64_t blocks = (M + kLdsBM - 1) / kLdsBM;
    if (g_tile_buffers == 1)
        hipLaunchKernelGGL((linear_kernel<V, NT, 1>), dim3((unsigned)blocks), dim3(256), 0, s, X,
                           ldx, W, b, Y, ldy, M, K, C);
    else
        hipLaunchKernelGGL((linear_kernel<V, NT, 2>), dim3((unsigned)blocks), dim3(256), 0, s, X,
                           ldx, W, b, Y, ldy, M, K, C);
    return hipGetLastError();
}

template <int V>
hipError_t dispatch_nt(int nt, const float *X, int64_t ldx, const float *W, const float *b,
                       float *Y, int64_t ldy, int M, int K, int C, hipStream_t s) {
    switch (nt) {
        case 1: return launch_linear<V, 1>(X, ldx, W, b, Y, ldy, M, K, C, s);
        case 2: return launch_linear<V, 2>(X, ldx, W, b, Y, ldy, M, K, C, s);
        case 3: return launch_linear<V, 3>(X, ldx, W, b, Y, ldy, M, K, C, s);
        case 4: return launch_linear<V, 4>(X, ldx, W, b, Y, ldy, M, K, C, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

// The current device's CU count, and the 160 KB dynamic-LDS attribute of a
// persistent kernel raised once per (device, kernel): both kept per device
// under a lock (a process may launch on several devices, from several threads).
hipError_t persistent_setup(const void *kernel, int *cus) {
    static std::mutex mu;
    static std::map<int, int> cu_count;
    static std::set<std::pair<int, const void *>> raised;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cu_count.find(dev);
    if (it == cu_count.end()) {
        int n = 0;
        e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        it = cu_count.emplace(dev, n).first;
    }
    *cus = it->second;
    if (!raised.count({dev, kernel})) {
        e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        raised.insert({dev, kernel});
    }
    return hipSuccess;
}

template <int V, int NT, int DIAG = 0, int CK = 32>
hipError_t launch_stream(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                         int64_t ldy, int M, int K, int C, int Kp, size_t lds, hipStream_t s) {
    int cus = 0;
    hipError_t e = persistent_setup(
        reinterpret_cast<const void *>(&linear_stream_kernel<V, NT, DIAG, CK>), &cus);
    if (e != hipSuccess) return e;
    // one workgroup per CU, at most one per tile
    const int tiles = (M + 15) / 16;
    const int blocks = std::max(1, std::min(cus, tiles));
    hipLaunchKernelGGL((linear_stream_kernel<V, NT, DIAG, CK>), dim3((unsigned)blocks),
                       dim3(64 * kStreamWaves), lds, s, X, ldx, W, b, Y, ldy, M, K, C, Kp);
    return hipGetLastError();
}

#ifndef SGC_SPLIT_WAVES
#define SGC_SPLIT_WAVES 8
#endif
// waves of the one workgroup per CU: 8 (12 or 16 measured 0.145 / 0.138 vs
// 0.089 ms: the register budget at 3-4 waves per SIMD spills the ring,
// profiles/r05/linear_ab_waves.log)
constexpr int kSplitWaves = SGC_SPLIT_WAVES;

// Split-bf16 kernel: W's operand image (split_chunk_bytes per 32-k chunk) +
// the tile counter.
inline size_t split_lds(int64_t K, int C) {
    const int NT = (C + 15) / 16;
    return (size_t)((K + 31) / 32) * split_chunk_bytes(NT, C - (NT - 1) * 16) + 16;
}

bool split_fits(int64_t M, int64_t K, int64_t ldx, int64_t ldy, int C) {
    return split_lds(K, C) <= 160 * 1024 && M * ldx * 4 < INT32_MAX && M * ldy * 4 < INT32_MAX &&
           K * C < (int64_t(1) << 29);
}

template <int NT, int DIAG>
hipError_t launch_split(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                        int64_t ldy, int M, int K, int C, hipStream_t s) {
    int cus = 0;
    hipError_t e = persistent_setup(
        reinterpret_cast<const void *>(&linear_split_kernel<NT, kSplitWaves, DIAG>), &cus);
    if (e != hipSuccess) return e;
    const int tiles = (M + 15) / 16;
    const int blocks = std::max(1, std::min(cus, tiles));
    hipLaunchKernelGGL((linear_split_kernel<NT, kSplitWaves, DIAG>), dim3((unsigned)blocks),
                       dim3(64 * kSplitWaves), split_lds(K, C), s, X, ldx, W, b, Y, ldy, M, K, C);
    return hipGetLastError();
}

// Streaming kernel preconditions: W's image within LDS, X within 31-bit byte
// offsets, rows 8-B aligned.
bool stream_fits(int64_t M, int64_t K, int64_t ldx, int nt, const float *X, size_t *lds) {
    *lds = (size_t)nt * 16 * ((K + 63) / 64 * 64) * 4 + 16;  // + the tile counter
    return *lds <= 160 * 1024 && M * ldx * 4 < INT32_MAX && ldx % 2 == 0 &&
           reinterpret_cast<uintptr_t>(X) % 8 == 0;
}

// Which forward kernel a class block of cc <= 64 classes takes (the
// diagnostic forms, tuning 3 / 4 / 6, count as their kernel).
enum LinearChoice { kLinTile, kLinStream, kLinSplit };
LinearChoice linear_choice(int64_t M, int64_t K, int64_t ldx, int64_t ldy, int cc,
                           const float *X) {
    size_t lds = 0;
    const bool stream_ok = stream_fits(M, K, ldx, (cc + 15) / 16, X, &lds);
    const bool split_ok = split_fits(M, K, ldx, ldy, cc);
    if (g_linear_kernel >= 5 || (g_linear_kernel == 0 && split_ok && M >= 4096)) return kLinSplit;
    if (g_linear_kernel >= 2 || (g_linear_kernel == 0 && stream_ok && M >= 4096)) return kLinStream;
    return kLinTile;
}

const char *linear_kernel_name(int64_t M, int64_t K, int64_t ldx, int64_t C, const float *X) {
    static const char *names[] = {
        "linear_kernel (LDS tile, v_mfma_f32_16x16x4_f32)",
        "linear_stream_kernel (fp32 streaming, v_mfma_f32_16x16x4_f32)",
        "linear_split_kernel (split-bf16 streaming, v_mfma_f32_16x16x32_bf16 x 6 products)"};
    if (M <= 0 || K <= 0 || C <= 0 || ldx < K) return "none";
    return names[linear_choice(M, K, ldx, C, (int)std::min<int64_t>(C, 64), X)];
}

int launch_linear_f32(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                      int64_t ldy, int64_t M, int64_t K, int64_t C, hipStream_t stream) {
    SGC_REQUIRE(X && W && Y, SGC_EINVAL, "linear: null pointer");
    SGC_REQUIRE(M >= 0 && K > 0 && C > 0 && ldx >= K && ldy >= C, SGC_EINVAL,
                "linear: bad shape M=%lld K=%lld C=%lld ldx=%lld ldy=%lld", (long long)M,
                (long long)K, (long long)C, (long long)ldx, (long long)ldy);
    SGC_REQUIRE(M < INT32_MAX && K < INT32_MAX, SGC_ERANGE, "linear: too large");
    SGC_REQUIRE(block_tile_fits(ldx, K, std::min<int64_t>(C, 64)), SGC_ERANGE,
                "linear: ldx=%lld / K=%lld past the tile's 31-bit offsets", (long long)ldx,
                (long long)K);
    if (M == 0) return SGC_OK;
    // classes are processed 64 at a time (NT <= 4 tiles of 16)
    for (int64_t c0 = 0; c0 < C; c0 += 64) {
        const int cc = (int)std::min<int64_t>(64, C - c0);
        const int nt = (cc + 15) / 16;
        const float *Wc = W + c0 * K;
        const float *bc = b ? b + c0 : nullptr;
        float *Yc = Y + c0;
        size_t lds = 0;
        const bool stream_ok = stream_fits(M, K, ldx, nt, X, &lds);
        const bool split_ok = split_fits(M, K, ldx, ldy, cc);
        if (linear_choice(M, K, ldx, ldy, cc, X) == kLinSplit) {
            SGC_REQUIRE(split_ok, SGC_EINVAL, "linear: split kernel preconditions not met");
            hipError_t e;
            const int diag = g_linear_kernel - 5;
#define SGC_SPLIT_NT(NTV)                                                                       \
    (diag == 1 ? launch_split<NTV, 1>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, stream)    \
     : diag == 2 ? launch_split<NTV, 2>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, stream)  \
     : diag == 3 ? launch_split<NTV, 3>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, stream)  \
                 : launch_split<NTV, 0>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, stream))
            switch (nt) {
                case 1: e = SGC_SPLIT_NT(1); break;
                case 2: e = SGC_SPLIT_NT(2); break;
                case 3: e = SGC_SPLIT_NT(3); break;
                default: e = SGC_SPLIT_NT(4); break;
            }
#undef SGC_SPLIT_NT
            SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "linear launch failed: %s", hipGetErrorString(e));
            continue;
        }
        if (g_linear_kernel >= 3) {  // diagnostics: NT = 3, 8-B rows only
            SGC_REQUIRE(stream_ok && nt == 3, SGC_EINVAL, "linear: diagnostic kernel needs NT = 3");
            const int Kp = (int)((K + 31) / 32 * 32);
            hipError_t e = g_linear_kernel == 3
                ? launch_stream<2, 3, 1>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, Kp, lds, stream)
                : launch_stream<2, 3, 2>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, Kp, lds, stream);
            SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "linear launch failed: %s", hipGetErrorString(e));
            continue;
        }
        if (linear_choice(M, K, ldx, ldy, cc, X) == kLinStream) {
            SGC_REQUIRE(stream_ok, SGC_EINVAL, "linear: streaming kernel preconditions not met");
            const int Kp = (int)((K + 31) / 32 * 32);
            const bool v4 = ldx % 4 == 0 && reinterpret_cast<uintptr_t>(X) % 16 == 0;
            hipError_t e;
            const int Kp64 = (int)((K + 63) / 64 * 64);
#define SGC_STREAM_NT(VV, NTV)                                                                  \
    (g_linear_ck == 64                                                                          \
         ? launch_stream<VV, NTV, 0, 64>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, Kp64, lds, stream) \
         : launch_stream<VV, NTV, 0, 32>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, Kp, lds, stream))
#define SGC_STREAM(VV)                                  \
    switch (nt) {                                       \
        case 1: e = SGC_STREAM_NT(VV, 1); break;        \
        case 2: e = SGC_STREAM_NT(VV, 2); break;        \
        case 3: e = SGC_STREAM_NT(VV, 3); break;        \
        default: e = SGC_STREAM_NT(VV, 4); break;       \
    }
            if (v4) {
                SGC_STREAM(4)
            } else {
                SGC_STREAM(2)
            }
#undef SGC_STREAM
#undef SGC_STREAM_NT
            SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "linear launch failed: %s", hipGetErrorString(e));
            continue;
        }
        int V = 1;
        for (int v : {4, 2}) {
            // natural alignment of every vector load (the k >= K tail is masked)
            if (K % v == 0 && ldx % v == 0 && reinterpret_cast<uintptr_t>(X) % (4 * v) == 0 &&
                reinterpret_cast<uintptr_t>(Wc) % (4 * v) == 0) {
                V = v;
                break;
            }
        }
        hipError_t e;
        if (V == 4)
            e = dispatch_nt<4>(nt, X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, stream);
        else if (V == 2)
            e = dispatch_nt<2>(nt, X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, stream);
        else
            e = dispatch_nt<1>(nt, X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, stream);
        SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "linear launch failed: %s", hipGetErrorString(e));
    }
    return SGC_OK;
}

SGC_WARM_UNIT(warm_linear)

}  // namespace sgc
