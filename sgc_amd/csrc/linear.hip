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
