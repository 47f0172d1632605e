// linear.hip -- SGC classifier forward  Y = X . W^T + b  (reference
// models.py:17-18: nn.Linear(nfeat, nclass)) on gfx950 fp32 MFMA.
//
// v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf chain per output,
// cdna_hip_programming.md 3) -- lane l holds A[l&15][l>>4], B[l>>4][l&15],
// D[4*(l>>4)+r][l&15].  A = 16 rows of X, B = 16 classes of W^T.
//
// Each lane loads V consecutive k of one X row (and of one W row) per step,
// so one step covers 4V values of k with V MFMAs; MFMA v sums k = k0+g*V+v
// over the lane groups g = 0..3.  A wave owns MT x 16 rows and all classes
// (NT x 16, padded), so X is read exactly once from HBM; W (nclass x nfeat,
// 99 KB at Reddit shape) is re-read per wave from L2.  At the Reddit-train
// shape the fp32 MFMA work (2 x 152,410 x 602 x 48 = 8.8 GFLOP, 56 us at
// 157 TF) and the X read (367 MB, ~60 us) are about even.
#include "gemm_tile.h"

namespace sgc {

template <int V, int MT, int NT>
__global__ __launch_bounds__(256) void linear_kernel(const float *__restrict__ X, int64_t ldx,
                                                     const float *__restrict__ W,
                                                     const float *__restrict__ b,
                                                     float *__restrict__ Y, int64_t ldy, int M,
                                                     int K, int C) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int m0 = wave * (MT * 16);
    if (m0 >= M) return;
    const int i = lane & 15, g = lane >> 4;

    const float *xrow[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        const int m = min(m0 + t * 16 + i, M - 1);
        xrow[t] = X + (int64_t)m * ldx;
    }
    const float *wrow[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int c = min(n * 16 + i, C - 1);
        wrow[n] = W + (int64_t)c * K;
    }
    f32x4 acc[MT][NT];
    xwt_tile<V, MT, NT>(xrow, wrow, K, g, acc);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int c = n * 16 + i;
        if (c >= C) continue;
        const float bias = b ? b[c] : 0.0f;
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + t * 16 + g * 4 + r;
                if (m < M) Y[(int64_t)m * ldy + c] = acc[t][n][r] + bias;
            }
    }
}

namespace {

template <int V, int MT, int NT>
hipError_t launch_linear(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                         int64_t ldy, int M, int K, int C, hipStream_t s) {
    const int rows_per_wave = MT * 16;
    const int64_t waves = (M + rows_per_wave - 1) / rows_per_wave;
    const int64_t blocks = (waves + 3) / 4;
    hipLaunchKernelGGL((linear_kernel<V, MT, NT>), dim3((unsigned)blocks), dim3(256), 0, s, X, ldx,
                       W, b, Y, ldy, M, K, C);
    return hipGetLastError();
}

template <int V>
hipError_t dispatch_nt(int nt, const float *X, int64_t ldx, const float *W, const float *b,
                       float *Y, int64_t ldy, int M, int K, int C, hipStream_t s) {
    switch (nt) {
        case 1: return launch_linear<V, 2, 1>(X, ldx, W, b, Y, ldy, M, K, C, s);
        case 2: return launch_linear<V, 2, 2>(X, ldx, W, b, Y, ldy, M, K, C, s);
        case 3: return launch_linear<V, 2, 3>(X, ldx, W, b, Y, ldy, M, K, C, s);
        case 4: return launch_linear<V, 2, 4>(X, ldx, W, b, Y, ldy, M, K, C, s);
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

}  // namespace sgc
