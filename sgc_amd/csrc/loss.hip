// loss.hip -- softmax cross-entropy over a logits matrix on gfx950: what the
// reference's training closures compute after the classifier,
//     loss = F.cross_entropy(model(x), y); loss.backward()
// (citation.py:46-49, reddit.py:55-58; mean reduction, ignore_index rows
// left out of the mean).  torch's CUDA/HIP form of that loss spends its time
// in a one-workgroup nll reduction (212 us forward + 131 us backward at the
// Reddit-train shape, 152,410 x 41 logits, profiles/r04/final3/kernel_stats.csv)
// for 25 MB of logits; here it is two passes over them.
//
//   ce_fwd_kernel     16 lanes per row (4 rows per wave, classes l, l+16, l+32,
//                     l+48 per lane, so C <= 64): row max and sum of exp by
//                     xor shuffles inside the 16-lane group, lse[row] stored,
//                     (lse - y[label]) summed in double per workgroup with the
//                     count of counted rows -> one partial per workgroup;
//   ce_finish_kernel  the partials in a fixed order (deterministic run to
//                     run): loss = sum / count and 1 / count;
//   ce_bwd_kernel     dY = (exp(Y - lse) - onehot(y)) * grad * (1 / count),
//                     zero rows for ignored labels.
// A label outside [0, C) (and not ignore_index) makes the loss NaN (torch
// stops with a device assert there).
#include <algorithm>
#include <cmath>

#include "common.h"

namespace sgc {

namespace {

constexpr int kCeRowsPerBlock = 16;  // 4 waves x 4 rows
constexpr int kCeMaxBlocks = 4096;

__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 16));
    return v;
}

__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
    return v;
}

__global__ __launch_bounds__(256) void ce_fwd_kernel(const float *__restrict__ Y, int64_t ldy,
                                                     const int64_t *__restrict__ labels, int M,
                                                     int C, int64_t ignore_index,
                                                     float *__restrict__ lse,
                                                     double *__restrict__ part_loss,
                                                     int *__restrict__ part_cnt) {
    __shared__ double red[256];
    __shared__ int redc[256];
    const int l = threadIdx.x & 15;
    const int g = threadIdx.x >> 4;  // row group of the block, 0..15
    double acc = 0.0;
    int cnt = 0;
    for (int64_t row = (int64_t)blockIdx.x * kCeRowsPerBlock + g; row < M;
         row += (int64_t)gridDim.x * kCeRowsPerBlock) {
        const float *yr = Y + row * ldy;
        float v[4];
        float m = -INFINITY;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = l + 16 * q;
            v[q] = c < C ? yr[c] : -INFINITY;
            m = fmaxf(m, v[q]);
        }
        m = group16_max(m);
        float s = 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (l + 16 * q < C) s += expf(v[q] - m);
        s = group16_sum(s);
        const float L = m + logf(s);
        const int64_t y = labels[row];
        if (l == 0) {
            lse[row] = L;
            if (y != ignore_index) {
                const float yv = (y >= 0 && y < C) ? yr[y] : NAN;
                acc += (double)(L - yv);
                ++cnt;
            }
        }
    }
    red[threadIdx.x] = acc;
    redc[threadIdx.x] = cnt;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) {
            red[threadIdx.x] += red[threadIdx.x + h];
            redc[threadIdx.x] += redc[threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part_loss[blockIdx.x] = red[0];
        part_cnt[blockIdx.x] = redc[0];
    }
}

// out[0] = loss (mean over the counted rows), out[1] = 1 / count.
__global__ __launch_bounds__(256) void ce_finish_kernel(const double *__restrict__ part_loss,
                                                        const int *__restrict__ part_cnt, int nb,
                                                        float *__restrict__ loss,
                                                        float *__restrict__ inv_count) {
    __shared__ double red[256];
    __shared__ long long redc[256];
    double s = 0.0;
    long long c = 0;
    for (int j = threadIdx.x; j < nb; j += 256) {
        s += part_loss[j];
        c += part_cnt[j];
    }
    red[threadIdx.x] = s;
    redc[threadIdx.x] = c;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) {
            red[threadIdx.x] += red[threadIdx.x + h];
            redc[threadIdx.x] += redc[threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        // count 0: 0 / 0 = NaN, as torch's mean over no rows
        *loss = (float)(red[0] / (double)redc[0]);
        *inv_count = (float)(1.0 / (double)redc[0]);
    }
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(const float *__restrict__ Y, int64_t ldy,
                                                     const int64_t *__restrict__ labels,
                                                     const float *__restrict__ lse,
                                                     const float *__restrict__ inv_count,
                                                     const float *__restrict__ grad, int M, int C,
                                                     int64_t ignore_index, float *__restrict__ dY,
                                                     int64_t lddy) {
    const int l = threadIdx.x & 15;
    const int g = threadIdx.x >> 4;
    const float scale = (grad ? *grad : 1.0f) * *inv_count;
    for (int64_t row = (int64_t)blockIdx.x * kCeRowsPerBlock + g; row < M;
         row += (int64_t)gridDim.x * kCeRowsPerBlock) {
        const float *yr = Y + row * ldy;
        float *dr = dY + row * lddy;
        const int64_t y = labels[row];
        const bool ign = y == ignore_index;
        const float L = lse[row];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = l + 16 * q;
            if (c < C) dr[c] = ign ? 0.0f : (expf(yr[c] - L) - (c == y ? 1.0f : 0.0f)) * scale;
        }
    }
}

int ce_blocks(int64_t M) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(kCeMaxBlocks,
                                                       (M + kCeRowsPerBlock - 1) / kCeRowsPerBlock));
}

}  // namespace

int64_t cross_entropy_workspace(int64_t M, int64_t C) {
    (void)C;
    return M <= 0 ? 0 : (int64_t)ce_blocks(M) * 16 + 256;
}

int cross_entropy_fwd_f32(const float *Y, int64_t ldy, const int64_t *labels, int64_t M, int64_t C,
                          int64_t ignore_index, float *loss, float *inv_count, float *lse, void *ws,
                          int64_t ws_bytes, hipStream_t s) {
    SGC_REQUIRE(Y && labels && loss && inv_count && lse && ws, SGC_EINVAL,
                "cross_entropy: null pointer");
    SGC_REQUIRE(M > 0 && M < INT32_MAX && C > 0 && C <= 64 && ldy >= C, SGC_EINVAL,
                "cross_entropy: bad shape M=%lld C=%lld ldy=%lld (0 < C <= 64)", (long long)M,
                (long long)C, (long long)ldy);
    SGC_REQUIRE(ws_bytes >= cross_entropy_workspace(M, C), SGC_ENOMEM,
                "cross_entropy: workspace %lld < %lld", (long long)ws_bytes,
                (long long)cross_entropy_workspace(M, C));
    const int nb = ce_blocks(M);
    char *p = (char *)(((uintptr_t)ws + 15) & ~uintptr_t(15));
    double *part_loss = (double *)p;
    int *part_cnt = (int *)(p + (int64_t)nb * 8);
    hipLaunchKernelGGL(ce_fwd_kernel, dim3(nb), dim3(256), 0, s, Y, ldy, labels, (int)M, (int)C,
                       ignore_index, lse, part_loss, part_cnt);
    hipLaunchKernelGGL(ce_finish_kernel, dim3(1), dim3(256), 0, s, part_loss, part_cnt, nb, loss,
                       inv_count);
    const hipError_t e = hipGetLastError();
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "cross_entropy launch failed: %s", hipGetErrorString(e));
    return SGC_OK;
}

int cross_entropy_bwd_f32(const float *Y, int64_t ldy, const int64_t *labels, const float *lse,
                          const float *inv_count, const float *grad, int64_t M, int64_t C,
                          int64_t ignore_index, float *dY, int64_t lddy, hipStream_t s) {
    SGC_REQUIRE(Y && labels && lse && inv_count && dY, SGC_EINVAL,
                "cross_entropy_bwd: null pointer");
    SGC_REQUIRE(M > 0 && M < INT32_MAX && C > 0 && C <= 64 && ldy >= C && lddy >= C, SGC_EINVAL,
                "cross_entropy_bwd: bad shape M=%lld C=%lld (0 < C <= 64)", (long long)M,
                (long long)C);
    hipLaunchKernelGGL(ce_bwd_kernel, dim3(ce_blocks(M)), dim3(256), 0, s, Y, ldy, labels, lse,
                       inv_count, grad, (int)M, (int)C, ignore_index, dY, lddy);
    const hipError_t e = hipGetLastError();
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "cross_entropy_bwd launch failed: %s",
                hipGetErrorString(e));
    return SGC_OK;
}

SGC_WARM_UNIT(warm_loss)

}  // namespace sgc
