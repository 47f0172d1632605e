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
    VT xa[MT], wb[NT], xn[MT], wn[NT];
    auto load = [&](int k0, VT (&xd)[MT], VT (&wd)[NT]) {
        const int k = k0 + g * V;
        const bool ok = k < K;
        const int kk = ok ? k : 0;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            xd[t] = *reinterpret_cast<const VT *>(xrow[t] + kk);
            if (!ok) xd[t] = VT{};
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            wd[n] = *reinterpret_cast<const VT *>(wrow[n] + kk);
            if (!ok) wd[n] = VT{};
        }
    };
    load(0, xa, wb);
    for (int k0 = 0; k0 < K; k0 += 4 * V) {
        if (k0 + 4 * V < K) load(k0 + 4 * V, xn, wn);
#pragma unroll
        for (int v = 0; v < V; ++v)
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[t][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        lane_elem<V>(xa[t], v), lane_elem<V>(wb[n], v), acc[t][n], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < MT; ++t) xa[t] = xn[t];
#pragma unroll
        for (int n = 0; n < NT; ++n) wb[n] = wn[n];
    }
}

}  // namespace sgc
