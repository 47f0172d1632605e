// Micro-benchmark: the issue rate of v_mfma_f32_16x16x4_f32 on gfx950 in the
// classifier's pattern -- NT independent accumulators per wave, the A operand
// shared by the NT MFMAs of a k step, B from registers -- with W waves per
// SIMD and nothing else in the loop.  Built and run by hand:
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/mfma_rate.hip -o variants/mfma_rate
//   variants/mfma_rate
// Prints, per (NT, waves per SIMD): ms, MFMAs per SIMD, cycles per MFMA at the
// measured clock-free rate, and TFLOP/s (2 x 16 x 16 x 4 flops per MFMA).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

template <int NT>
__global__ __launch_bounds__(1024) void mfma_loop(float *out, int iters, float seed) {
    f32x4 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    float a[8], b[NT][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] = seed * (threadIdx.x + k);
#pragma unroll
        for (int n = 0; n < NT; ++n) b[n][k] = seed * (n + k + 1);
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[kk], b[n][kk], acc[n], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int n = 0; n < NT; ++n) s += acc[n][0] + acc[n][1] + acc[n][2] + acc[n][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NT>
void run(int cus, int waves_per_simd, int iters) {
    const int threads = 64 * 4 * waves_per_simd;  // one workgroup per CU
    float *d;
    CHECK(hipMalloc(&d, (size_t)cus * threads * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(mfma_loop<NT>, dim3(cus), dim3(threads), 0, 0, d, iters, 1e-3f);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(mfma_loop<NT>, dim3(cus), dim3(threads), 0, 0, d, iters, 1e-3f);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double per_simd = (double)iters * 8 * NT * waves_per_simd;  // MFMAs per SIMD
    const double total = per_simd * 4 * cus;
    printf("{\"NT\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"mfma_per_simd\": %.0f, "
           "\"ns_per_mfma_per_simd\": %.3f, \"TFLOPs\": %.1f}\n",
           NT, waves_per_simd, ms, per_simd, ms * 1e6 / per_simd, total * 2048.0 / ms / 1e9);
    CHECK(hipFree(d));
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    for (int w : {1, 2, 4}) {
        run<3>(cus, w, 20000 / w);
        run<2>(cus, w, 30000 / w);
        run<6>(cus, w, 10000 / w);
    }
    return 0;
}
