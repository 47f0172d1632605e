// Micro-benchmark: writing the classifier's output Y [M, C] fp32 (row pitch C
// = 41 at the Reddit-train shape: rows 4-B aligned) per 16-row tile in the
// shapes the forward kernels could use, alone (no loads).
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/store_shape.hip -o variants/store_shape
//   variants/store_shape M C reps
// Modes, per 16-row tile per wave:
//   0  the split kernel's MFMA layout (D = W . X^T): lane (j, kg) writes classes
//      16n + 4kg .. +3 of row j -- one b128 per class tile (16 rows x 64 B each)
//   1  the fp32 kernels' layout: lane (i, g) writes class 16n + i of rows 4g..4g+3
//      -- four b32 per class tile
//   2  the tile's C x 16 floats as one contiguous run, 1 KB per b128 instruction
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0x80000000u;

template <int MODE>
__global__ __launch_bounds__(256) void store(float *Y, int M, int C) {
    const int lane = threadIdx.x & 63;
    const int j = lane & 15, kg = lane >> 4;
    const long long gw = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long nw = (long long)gridDim.x * 4;
    const int tiles = (M + 15) / 16;
    const auto yd = __builtin_amdgcn_make_buffer_rsrc(Y, 0, (int)((long long)M * C * 4), 0x00020000);
    const int NT = (C + 15) / 16;
    for (long long t = gw; t < tiles; t += nw) {
        const uint32_t v = (uint32_t)t;
        if constexpr (MODE == 0) {
            const uint32_t yrow = (uint32_t)((t * 16 + j) * C * 4);
            for (int n = 0; n < NT; ++n) {
                const int cl0 = n * 16 + 4 * kg;
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{v, v, v, v}, yd,
                                                       cl0 + 4 <= C ? yrow + 4u * cl0 : kOOB, 0, 0);
                if (cl0 < C && cl0 + 4 > C)
                    for (int r = 0; r < C - cl0; ++r)
                        __builtin_amdgcn_raw_buffer_store_b32(v, yd, yrow + 4u * (cl0 + r), 0, 0);
            }
        } else if constexpr (MODE == 1) {
            for (int n = 0; n < NT; ++n) {
                const int cl = n * 16 + j;
                for (int r = 0; r < 4; ++r) {
                    const uint32_t row = (uint32_t)(t * 16 + 4 * kg + r);
                    __builtin_amdgcn_raw_buffer_store_b32(v, yd, cl < C ? (row * C + cl) * 4u : kOOB,
                                                          0, 0);
                }
            }
        } else {
            const uint32_t base = (uint32_t)(t * 16 * C * 4);
            const int bytes = 16 * C * 4;
            for (int o = lane * 16; o < bytes; o += 1024)
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{v, v, v, v}, yd,
                                                       o + 16 <= bytes ? base + o : kOOB, 0, 0);
        }
    }
}

template <int MODE>
float run(float *Y, int M, int C, int blocks, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((store<MODE>), dim3(blocks), dim3(256), 0, 0, Y, M, C);
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((store<MODE>), dim3(blocks), dim3(256), 0, 0, Y, M, C);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 152410;
    const int C = argc > 2 ? atoi(argv[2]) : 41;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    float *Y;
    CHECK(hipMalloc(&Y, (size_t)M * C * 4));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const double bytes = (double)M * C * 4;
    for (int bpc : {2, 8}) {
        const int blocks = cus * bpc;
        const float t0 = run<0>(Y, M, C, blocks, reps), t1 = run<1>(Y, M, C, blocks, reps),
                    t2 = run<2>(Y, M, C, blocks, reps);
        printf("M=%d C=%d waves/CU=%d  mfma-T b128 %.4f ms %.2f TB/s | fp32 b32 %.4f ms %.2f TB/s | "
               "flat b128 %.4f ms %.2f TB/s\n",
               M, C, bpc * 4, t0, bytes / t0 / 1e9, t1, bytes / t1 / 1e9, t2, bytes / t2 / 1e9);
    }
    return 0;
}
