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
