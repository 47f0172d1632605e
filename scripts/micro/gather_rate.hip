// Micro-benchmark: the chip's rate of gathering row SEGMENTS (one row of X,
// W floats, read by W/4 lanes of 16 B) in the SpMM's access order, with no
// CSR walk, no LDS staging and no FMA chain -- what a narrow SpMM pass could
// reach if nothing but the gathers cost.  Built and run by hand:
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/gather_rate.hip -o variants/gather_rate
//   variants/gather_rate cols.bin reps width:ld:mode:group_lanes ...
// cols.bin: int32 column ids in CSR order (scripts/micro/gather_cols.py).
// Each wave holds R = 64 / LR row groups of LR lanes; group g walks a run of
// kRun consecutive nonzeros (its "row"), U gathers in flight per step, two
// steps pipelined.  The byte offsets are precomputed (col * ld * 4) and read
// four at a time (one 16-B load, the same address in every lane of a group).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef int i4 __attribute__((ext_vector_type(4)));
constexpr int kRun = 64;  // nonzeros per group (a light row of the Reddit shape)

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

template <int U>
__global__ __launch_bounds__(256) void gather(const int *__restrict__ off, long long nnz,
                                              const float *__restrict__ X, int LR, int active,
                                              float *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int R = 64 / LR;
    const int g = min(lane / LR, R - 1);  // lanes past R*LR duplicate the last group
    // lanes of a group past `active` read the row's first 16 B (as the
    // heavy-row pairs path's idle lanes do)
    const int l = (lane - (lane / LR) * LR) < active ? lane - (lane / LR) * LR : 0;
    const long long wave = (long long)blockIdx.x * 4 + threadIdx.x / 64;
    const long long run = wave * R + g;
    const long long k0 = run * kRun;
    if (k0 >= nnz) return;  // (ragged last wave: groups past the end idle)
    const char *Xb = reinterpret_cast<const char *>(X);
    const uint32_t boff = (uint32_t)l * 16u;
    f4 acc = {0, 0, 0, 0};
    const i4 *o4 = reinterpret_cast<const i4 *>(off + k0);
    f4 xv[2][U];
#pragma unroll
    for (int q = 0; q < U / 4; ++q) {
        const i4 c = o4[q];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            xv[0][4 * q + u] = *reinterpret_cast<const f4 *>(Xb + (uint32_t)(c[u] + boff));
    }
#pragma unroll
    for (int s = 0; s < kRun / U; ++s) {
        if (s + 1 < kRun / U) {
#pragma unroll
            for (int q = 0; q < U / 4; ++q) {
                const i4 c = o4[(s + 1) * (U / 4) + q];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    xv[(s + 1) & 1][4 * q + u] =
                        *reinterpret_cast<const f4 *>(Xb + (uint32_t)(c[u] + boff));
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += xv[s & 1][u];
    }
    out[wave * 64 + lane] = acc[0] + acc[1] + acc[2] + acc[3];
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s cols.bin [reps]\n", argv[0]);
        return 2;
    }
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    const long long nnz_all = ftell(f) / 4;
    fseek(f, 0, SEEK_SET);
    std::vector<int> col(nnz_all);
    if (fread(col.data(), 4, nnz_all, f) != (size_t)nnz_all) return 2;
    fclose(f);
    const int n = *std::max_element(col.begin(), col.end()) + 1;
    const long long nnz = nnz_all / kRun * kRun;
    printf("{\"n\": %d, \"nnz\": %lld}\n", n, nnz);
    int *d_off;
    float *d_out;
    CHECK(hipMalloc(&d_off, nnz * 4));
    CHECK(hipMalloc(&d_out, (nnz / kRun + 64) * 64 * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    struct Case {
        int width, ld, mode, group;  // mode 0: CSR order, 1: uniform random, 2: hot (2048 rows)
    };
    // cases from argv[3..]: "width:ld:mode:group_lanes" (group 0 = width / 4)
    std::vector<Case> cases;
    for (int i = 3; i < argc; ++i) {
        Case c{76, 96, 0, 0};
        sscanf(argv[i], "%d:%d:%d:%d", &c.width, &c.ld, &c.mode, &c.group);
        cases.push_back(c);
    }
    std::vector<int> off(nnz);
    srand(1);
    for (const Case &c : cases) {
        const int active = (c.width + 3) / 4;
        const int LR = c.group > 0 ? c.group : active;
        const int R = 64 / LR;
        for (long long k = 0; k < nnz; ++k) {
            int cj = col[k];
            if (c.mode == 1) cj = (int)(((unsigned long long)rand() * 2654435761ull) % n);
            if (c.mode == 2) cj = col[k] & 2047;
            off[k] = cj * c.ld * 4;
        }
        CHECK(hipMemcpy(d_off, off.data(), nnz * 4, hipMemcpyHostToDevice));
        float *d_x;
        CHECK(hipMalloc(&d_x, (size_t)n * c.ld * 4));
        CHECK(hipMemset(d_x, 0, (size_t)n * c.ld * 4));
        const long long runs = nnz / kRun;
        const long long waves = (runs + R - 1) / R;
        const unsigned blocks = (unsigned)((waves + 3) / 4);
        for (int U : {4, 8}) {
            auto launch = [&]() {
                if (U == 4)
                    hipLaunchKernelGGL(gather<4>, dim3(blocks), dim3(256), 0, 0, d_off, nnz, d_x,
                                       LR, active, d_out);
                else
                    hipLaunchKernelGGL(gather<8>, dim3(blocks), dim3(256), 0, 0, d_off, nnz, d_x,
                                       LR, active, d_out);
            };
            launch();
            CHECK(hipDeviceSynchronize());
            std::vector<float> ms;
            for (int r = 0; r < reps; ++r) {
                CHECK(hipEventRecord(e0, 0));
                launch();
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float t;
                CHECK(hipEventElapsedTime(&t, e0, e1));
                ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            const double t = ms[ms.size() / 2];
            const int lines = (c.width * 4 + 127) / 128;
            printf("{\"width\": %d, \"ld\": %d, \"mode\": %d, \"U\": %d, \"group_lanes\": %d, "
                   "\"rows_per_wave\": %d, "
                   "\"ms\": %.4f, \"Gseg_per_s\": %.2f, \"useful_TBps\": %.2f, "
                   "\"line_TBps\": %.2f}\n",
                   c.width, c.ld, c.mode, U, LR, R, t, nnz / t / 1e6, nnz * c.width * 4.0 / t / 1e9,
                   nnz * lines * 128.0 / t / 1e9);
            fflush(stdout);
        }
        CHECK(hipFree(d_x));
    }
    return 0;
}
