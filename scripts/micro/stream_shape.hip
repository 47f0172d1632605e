// Micro-benchmark: HBM read rate of the classifier's X stream (X [M, K] fp32,
// row pitch ldx) for different per-wave-instruction access shapes, every wave
// walking 16-row tiles as the streaming classifier kernel does.  Loads only:
// each lane sums what it reads (one store per lane at the end).
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/stream_shape.hip -o variants/stream_shape
//   variants/stream_shape M K ldx reps
// Modes (per 16-row tile, per chunk of the row):
//   0  the round-4 kernel's shape: lane (i, g) = (l & 15, l >> 4) reads row i,
//      8-B loads at 16g + {0, 8} + 64{0..3} of a 256-B chunk (8 loads / chunk)
//   1  8 lanes x 16 B per row, 8 rows per instruction: 128 contiguous bytes of
//      each row per instruction (2 loads per 128-B chunk of 16 rows)
//   2  16 lanes x 16 B per row, 4 rows per instruction (256 contiguous bytes;
//      4 loads per 256-B chunk)
//   3  flat: the tile's bytes as one contiguous run, 1 KB per instruction
//   4  mode 1 with 8-B loads: 16 lanes x 8 B per row, 4 rows per instruction
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__device__ __forceinline__ f4 ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ f2 ld2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

// U = chunks in flight per lane (loads issued before any is summed)
template <int MODE, int U>
__global__ __launch_bounds__(256) void stream(const float *__restrict__ X, int ldx, int M, int K,
                                              float *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int i = lane & 15, g = lane >> 4;
    const long long gw = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long nw = (long long)gridDim.x * 4;
    const int tiles = (M + 15) / 16;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(X), 0,
                                                      (int)((long long)M * ldx * 4), 0x00020000);
    const uint32_t pitch = (uint32_t)ldx * 4u;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long long t = gw; t < tiles; t += nw) {
        const uint32_t tb = (uint32_t)(t * 16) * pitch;
        if constexpr (MODE == 0) {
            const int nch = (K * 4 + 255) / 256;
            const uint32_t rb = tb + (uint32_t)i * pitch + 16u * g;
            for (int c = 0; c < nch; c += U) {
                f2 v[U][8];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        v[u][q] = (c + u < nch) ? ld2(rs, rb + (c + u) * 256u + ((q * 8) & 15) +
                                                                  ((q * 8) >> 4) * 64)
                                                : f2{0.f, 0.f};
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int q = 0; q < 8; ++q) acc[q & 3] += v[u][q][0] + v[u][q][1];
            }
        } else if constexpr (MODE == 1) {
            const int nch = (K * 4 + 127) / 128;
            const uint32_t seg = 16u * (2 * g + (i >> 3));
            const uint32_t r0 = tb + (uint32_t)(i & 7) * pitch + seg;
            for (int c = 0; c < nch; c += U) {
                f4 v[U][2];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        v[u][h] = (c + u < nch) ? ld4(rs, r0 + 8u * h * pitch + (c + u) * 128u)
                                                : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int u = 0; u < U; ++u) acc += v[u][0] + v[u][1];
            }
        } else if constexpr (MODE == 2) {
            const int nch = (K * 4 + 255) / 256;
            const uint32_t r0 = tb + (uint32_t)(lane >> 4) * pitch + 16u * (lane & 15);
            for (int c = 0; c < nch; c += U) {
                f4 v[U][4];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int h = 0; h < 4; ++h)
                        v[u][h] = (c + u < nch) ? ld4(rs, r0 + 4u * h * pitch + (c + u) * 256u)
                                                : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int u = 0; u < U; ++u) acc += v[u][0] + v[u][1] + v[u][2] + v[u][3];
            }
        } else if constexpr (MODE == 3) {
            const uint32_t bytes = 16u * pitch;
            const int nch = (bytes + 1023) / 1024;
            for (int c = 0; c < nch; c += 2 * U) {
                f4 v[2 * U];
#pragma unroll
                for (int u = 0; u < 2 * U; ++u)
                    v[u] = (c + u < nch) ? ld4(rs, tb + (c + u) * 1024u + 16u * lane)
                                         : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int u = 0; u < 2 * U; ++u) acc += v[u];
            }
        } else {
            const int nch = (K * 4 + 127) / 128;
            const uint32_t r0 = tb + (uint32_t)(lane >> 4) * pitch + 8u * (lane & 15);
            for (int c = 0; c < nch; c += U) {
                f2 v[U][4];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int h = 0; h < 4; ++h)
                        v[u][h] = (c + u < nch) ? ld2(rs, r0 + 4u * h * pitch + (c + u) * 128u)
                                                : f2{0.f, 0.f};
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int h = 0; h < 4; ++h) acc[h] += v[u][h][0] + v[u][h][1];
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <int MODE, int U>
float run(const float *X, int ldx, int M, int K, float *out, int blocks, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((stream<MODE, U>), dim3(blocks), dim3(256), 0, 0, X, ldx, M, K, out);
    CHECK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((stream<MODE, U>), dim3(blocks), dim3(256), 0, 0, X, ldx, M, K, out);
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
    const int K = argc > 2 ? atoi(argv[2]) : 602;
    const int ldx = argc > 3 ? atoi(argv[3]) : K;
    const int reps = argc > 4 ? atoi(argv[4]) : 20;
    const size_t n = (size_t)M * ldx;
    float *X, *out;
    CHECK(hipMalloc(&X, n * 4));
    CHECK(hipMemset(X, 0, n * 4));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const double bytes = (double)M * K * 4;
    for (int bpc : {2, 4, 8}) {
        const int blocks = cus * bpc;
        CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
        struct R { const char *name; float ms; } rs[] = {
            {"mode0 16x64B b64 (round 4)", run<0, 2>(X, ldx, M, K, out, blocks, reps)},
            {"mode1 8 rows x 128B b128 U2", run<1, 2>(X, ldx, M, K, out, blocks, reps)},
            {"mode1 8 rows x 128B b128 U4", run<1, 4>(X, ldx, M, K, out, blocks, reps)},
            {"mode2 4 rows x 256B b128 U2", run<2, 2>(X, ldx, M, K, out, blocks, reps)},
            {"mode3 flat 1KB b128 U2", run<3, 2>(X, ldx, M, K, out, blocks, reps)},
            {"mode4 4 rows x 128B b64 U4", run<4, 4>(X, ldx, M, K, out, blocks, reps)},
        };
        for (auto &r : rs)
            printf("M=%d K=%d ldx=%d waves/CU=%d %-30s %.4f ms  %.2f TB/s\n", M, K, ldx, bpc * 4,
                   r.name, r.ms, bytes / r.ms / 1e9);
        CHECK(hipFree(out));
    }
    return 0;
}
