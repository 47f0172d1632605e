// Micro-benchmark: issue rate of the bf16 MFMA shapes on gfx950 --
// v_mfma_f32_16x16x16_bf16 (k = 16: a lane holds 4 consecutive k of a column)
// vs v_mfma_f32_16x16x32_bf16 (k = 32) and v_mfma_f32_16x16x4_f32 -- with 12
// independent accumulators per wave, operands in registers, nothing else in
// the loop.  Decides whether the classifier's weight backward (reduction over
// rows) can take its 4-row-per-lane loads to bf16 MFMA without a transpose.
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/mfma_bf16_rate.hip -o variants/mfma_bf16_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int NA = 12;

template <int KIND>  // 0: 16x16x16 bf16, 1: 16x16x32 bf16, 2: 16x16x4 f32
__global__ __launch_bounds__(512) void loop(float *out, int iters, float seed) {
    f32x4 acc[NA];
#pragma unroll
    for (int n = 0; n < NA; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    const short sv = (short)(threadIdx.x * 7 + (int)seed);
    s16x4 a4 = {sv, (short)(sv + 1), (short)(sv + 2), (short)(sv + 3)};
    bf16x8 a8;
#pragma unroll
    for (int e = 0; e < 8; ++e) a8[e] = (__bf16)(seed * (threadIdx.x + e));
    float af = seed * threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int n = 0; n < NA; ++n) {
            if constexpr (KIND == 0)
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, a4, acc[n], 0, 0, 0);
            else if constexpr (KIND == 1)
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, a8, acc[n], 0, 0, 0);
            else
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(af, af, acc[n], 0, 0, 0);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int n = 0; n < NA; ++n) s += acc[n][0] + acc[n][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
void run(const char *name, int cus, int wps, int iters) {
    const int threads = 256 * wps;
    float *d;
    CHECK(hipMalloc(&d, (size_t)cus * threads * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(loop<KIND>, dim3(cus), dim3(threads), 0, 0, d, iters, 1.0f);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(loop<KIND>, dim3(cus), dim3(threads), 0, 0, d, iters, 1.0f);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double per_simd = (double)iters * NA * wps;
    printf("{\"mfma\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"ns_per_mfma_per_simd\": %.3f}\n",
           name, wps, ms, ms * 1e6 / per_simd);
    CHECK(hipFree(d));
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    for (int w : {1, 2}) {
        run<0>("16x16x16_bf16", cus, w, 20000);
        run<1>("16x16x32_bf16", cus, w, 20000);
        run<2>("16x16x4_f32", cus, w, 20000);
    }
    return 0;
}
