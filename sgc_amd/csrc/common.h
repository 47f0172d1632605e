// common.h -- shared helpers for the gfx950 kernels of libsgc_amd.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sgc_amd.h"

namespace sgc {

// Thread-local message for sgc_last_error().
void set_error(const char *fmt, ...);

#define SGC_HIP_CHECK(expr)                                                         \
    do {                                                                            \
        hipError_t _e = (expr);                                                     \
        if (_e != hipSuccess) {                                                     \
            ::sgc::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                             __FILE__, __LINE__);                                   \
            return SGC_EHIP;                                                        \
        }                                                                           \
    } while (0)

#define SGC_REQUIRE(cond, code, ...)       \
    do {                                   \
        if (!(cond)) {                     \
            ::sgc::set_error(__VA_ARGS__); \
            return (code);                 \
        }                                  \
    } while (0)

static constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// Code-object warm-up (sgc_warmup): the runtime loads a translation unit's
// code object on the first launch of any of its kernels, so one empty launch
// per unit moves that load out of the first real call.  SGC_WARM_UNIT(name)
// defines `hipError_t name(hipStream_t)` launching this unit's empty kernel.
#define SGC_WARM_UNIT(name)                                                 \
    namespace {                                                             \
    __global__ void name##_kernel() {}                                      \
    }                                                                       \
    hipError_t name(hipStream_t s) {                                        \
        hipLaunchKernelGGL(name##_kernel, dim3(1), dim3(kWave), 0, s);      \
        return hipGetLastError();                                           \
    }
hipError_t warm_spmm(hipStream_t);
hipError_t warm_side_streams();  // creates the SpMM's per-device side-stream pool
hipError_t warm_ingest(hipStream_t);
hipError_t warm_plan(hipStream_t);
hipError_t warm_sort(hipStream_t);
hipError_t warm_groups(hipStream_t);
hipError_t warm_exchange(hipStream_t);
hipError_t warm_linear(hipStream_t);
hipError_t warm_xent(hipStream_t);
hipError_t warm_loss(hipStream_t);
hipError_t warm_normalize(hipStream_t);
hipError_t warm_subgraph(hipStream_t);

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// V consecutive fp32 in one lane: float / float2 / float4 register vectors,
// loaded with one global_load_dword{,x2,x4}.
// LDS image depth of the classifier tile (gemm_tile.h; linear.hip defines it,
// sgc_set_tuning("tile_buffers") sets it: 1 or 2).
extern int g_tile_buffers;
// Classifier forward kernel (linear.hip): 0 auto, 1 LDS tile, 2 streaming.
extern int g_linear_kernel;
// k per chunk of the streaming classifier kernel (32 or 64).
extern int g_linear_ck;
// Classifier weight backward: 0 auto, 1 fp32 MFMA slabs, 2 split-bf16 slabs (xent.hip).
extern int g_backward_kernel;

template <int V> struct Vec { typedef float __attribute__((ext_vector_type(V))) T; };
template <> struct Vec<1> { typedef float T; };

template <int V>
__device__ __forceinline__ float lane_elem(const typename Vec<V>::T &x, int i) { return x[i]; }
template <>
__device__ __forceinline__ float lane_elem<1>(const float &x, int) { return x; }

template <int V>
__device__ __forceinline__ void set_elem(typename Vec<V>::T &x, int i, float v) { x[i] = v; }
template <>
__device__ __forceinline__ void set_elem<1>(float &x, int, float v) { x = v; }

}  // namespace sgc
