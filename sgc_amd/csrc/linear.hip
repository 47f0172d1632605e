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
#include "gemm_tile.h"

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


// 0 = auto (streaming where W fits LDS and the rows are 8-B aligned), 1 = the
// LDS tile, 2 = streaming (3 / 4: its DIAG forms, wrong results by design).
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

template <int V, int NT, int DIAG = 0, int CK = 32>
hipError_t launch_stream(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                         int64_t ldy, int M, int K, int C, int Kp, size_t lds, hipStream_t s) {
    static int cus = 0;
    static bool attr[5] = {false, false, false, false, false};
    if (!cus) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
    }
    if (!attr[NT]) {
        hipError_t e = hipFuncSetAttribute(
            reinterpret_cast<const void *>(&linear_stream_kernel<V, NT, DIAG, CK>),
            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr[NT] = true;
    }
    // one workgroup per CU, at most one per tile
    const int tiles = (M + 15) / 16;
    const int blocks = std::max(1, std::min(cus, tiles));
    hipLaunchKernelGGL((linear_stream_kernel<V, NT, DIAG, CK>), dim3((unsigned)blocks),
                       dim3(64 * kStreamWaves), lds, s, X, ldx, W, b, Y, ldy, M, K, C, Kp);
    return hipGetLastError();
}

// Streaming kernel preconditions: W's image within LDS, X within 31-bit byte
// offsets, rows 8-B aligned.
bool stream_fits(int64_t M, int64_t K, int64_t ldx, int nt, const float *X, size_t *lds) {
    *lds = (size_t)nt * 16 * ((K + 63) / 64 * 64) * 4 + 16;  // + the tile counter
    return *lds <= 160 * 1024 && M * ldx * 4 < INT32_MAX && ldx % 2 == 0 &&
           reinterpret_cast<uintptr_t>(X) % 8 == 0;
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
        if (g_linear_kernel >= 3) {  // diagnostics: NT = 3, 8-B rows only
            SGC_REQUIRE(stream_ok && nt == 3, SGC_EINVAL, "linear: diagnostic kernel needs NT = 3");
            const int Kp = (int)((K + 31) / 32 * 32);
            hipError_t e = g_linear_kernel == 3
                ? launch_stream<2, 3, 1>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, Kp, lds, stream)
                : launch_stream<2, 3, 2>(X, ldx, Wc, bc, Yc, ldy, (int)M, (int)K, cc, Kp, lds, stream);
            SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "linear launch failed: %s", hipGetErrorString(e));
            continue;
        }
        if (g_linear_kernel == 2 || (g_linear_kernel == 0 && stream_ok && M >= 4096)) {
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
