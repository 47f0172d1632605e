// exchange.hip -- the data movement around the multi-GPU exchanges
// (sgc_amd.distributed): one launch copies a list of 2-D
// blocks between two row-major fp32 buffers.
//
// The replicated output of the partitioned sgc_precompute (every rank gets
// the whole X_K, as reference utils.py:92-97 returns it) arrives from RCCL as
// all_gather_into_tensor's [P x rows, ld] image -- rank q's column block of a
// row chunk at rows [q*rows, (q+1)*rows) -- and must land in X_K's columns
// [c_q, c_{q+1}); the line partition's tail arrives as [P x B, ld] row
// blocks.  One launch per chunk moves every rank's block (P launches of a
// strided copy each paid a ramp, ~0.05 ms apiece at Reddit shape).
//
// Segment s: dst[dst_row + i, dst_col + j] = src[src_row + i, src_col + j]
// for i < rows, j < cols.  Grid y = segment.  A segment is copied as one flat
// run of rows x cols/V vectors of V floats: lane t of the grid takes vectors
// t, t + T, ..., t + (U-1) T (T = the grid's threads), all U loads issued
// before the stores, so a wave-instruction always covers 64 consecutive
// vectors -- whole rows of a narrow block and the next rows after them --
// instead of one row per instruction with the lanes past the block's width
// idle (a 76-float block on 8-B lanes used 38 of 64 lanes: the round-5
// unpack ran at 3.1 TB/s).
#include <algorithm>
#include <cstring>

#include "common.h"

namespace sgc {

namespace {

constexpr int kMaxBlockSegs = 64;
constexpr int kCopyU = 4;  // vectors per lane in flight

struct CopySeg {
    int64_t src_off, dst_off;  // floats
    int32_t rows, cols;
};

struct CopyArgs {
    CopySeg seg[kMaxBlockSegs];
};

template <int V>
__global__ __launch_bounds__(256) void copy_blocks_kernel(const float *__restrict__ src,
                                                          int64_t lds, float *__restrict__ dst,
                                                          int64_t ldd, CopyArgs a) {
    using VT = typename Vec<V>::T;
    const CopySeg s = a.seg[blockIdx.y];
    const uint32_t cv = (uint32_t)s.cols / V;  // vectors per row
    const uint32_t total = (uint32_t)s.rows * cv;
    const uint32_t T = gridDim.x * blockDim.x;
    const float *sb = src + s.src_off;
    float *db = dst + s.dst_off;
    for (uint32_t base = blockIdx.x * blockDim.x + threadIdx.x; base < total; base += kCopyU * T) {
        VT v[kCopyU];
        int64_t doff[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const uint32_t idx = base + u * T;
            doff[u] = -1;
            if (idx < total) {
                const uint32_t r = idx / cv, c = idx - r * cv;
                v[u] = *reinterpret_cast<const VT *>(sb + r * lds + (int64_t)c * V);
                doff[u] = r * ldd + (int64_t)c * V;
            }
        }
#pragma unroll
        for (int u = 0; u < kCopyU; ++u)
            if (doff[u] >= 0) *reinterpret_cast<VT *>(db + doff[u]) = v[u];
    }
}

// ---------------------------------------------------------------------------
// Peer pulls over IPC-mapped memory (the replicated output without RCCL).
//
// Every rank computes its column block of a last-hop row chunk into a buffer
// its peers have mapped (hipIpcOpenMemHandle), then raises that chunk's
// ready flag to the call's sequence number; each rank waits until every
// peer's flag for the chunk reached it and pulls all P blocks straight into
// X_K's columns.  Flags: release stores at system scope (the L2's dirty
// lines written back first), acquire loads at system scope, one wave that
// polls with a sleep and gives up after a wall-clock bound (the error word is
// then set and the host raises: a lost peer never hangs the GPU).  The pulled
// bytes are read with system-coherent buffer loads (sc0 sc1): a peer's block
// is never served from this GPU's caches, whatever an earlier call left there.

constexpr int kMaxPullSegs = 16;
constexpr int kMaxWaitFlags = 64;

struct PullSeg {
    const float *src;  // (src_row, src_col) already applied
    int64_t lds;       // floats
    int64_t dst_off;   // floats
    int32_t rows, cols;
};

struct PullArgs {
    PullSeg seg[kMaxPullSegs];
};

struct WaitArgs {
    const int32_t *flag[kMaxWaitFlags];
};

template <int V>
__device__ __forceinline__ typename Vec<V>::T load_sys(__amdgpu_buffer_rsrc_t r, uint32_t off);
template <>
__device__ __forceinline__ Vec<4>::T load_sys<4>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(Vec<4>::T, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 17));
}
template <>
__device__ __forceinline__ Vec<2>::T load_sys<2>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(Vec<2>::T, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 17));
}
template <>
__device__ __forceinline__ float load_sys<1>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 17));
}

// Segment s = blockIdx.y: dst[dst_off + i*ldd + j] = src[i*lds + j], i < rows,
// j < cols, as copy_blocks_kernel's flat vector run (the host keeps every
// segment's source span below 2^31 bytes: 32-bit buffer offsets).
template <int V>
__global__ __launch_bounds__(256) void pull_blocks_kernel(float *__restrict__ dst, int64_t ldd,
                                                          PullArgs a) {
    using VT = typename Vec<V>::T;
    const PullSeg s = a.seg[blockIdx.y];
    const uint32_t cv = (uint32_t)s.cols / V;
    const uint32_t total = (uint32_t)s.rows * cv;
    const uint32_t T = gridDim.x * blockDim.x;
    const uintptr_t base = reinterpret_cast<uintptr_t>(s.src);
    const uint32_t bytes = (uint32_t)(((int64_t)(s.rows - 1) * s.lds + s.cols) * 4);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void *>(base), 0, (int)bytes, 0x00020000);
    float *db = dst + s.dst_off;
    for (uint32_t b0 = blockIdx.x * blockDim.x + threadIdx.x; b0 < total; b0 += kCopyU * T) {
        VT v[kCopyU];
        int64_t doff[kCopyU];
#pragma unroll
        for (int u = 0; u < kCopyU; ++u) {
            const uint32_t idx = b0 + u * T;
            doff[u] = -1;
            if (idx < total) {
                const uint32_t r = idx / cv, c = idx - r * cv;
                v[u] = load_sys<V>(rsrc, (uint32_t)((r * s.lds + (int64_t)c * V) * 4));
                doff[u] = r * ldd + (int64_t)c * V;
            }
        }
#pragma unroll
        for (int u = 0; u < kCopyU; ++u)
            if (doff[u] >= 0) *reinterpret_cast<VT *>(db + doff[u]) = v[u];
    }
}

// One wave: lane i < n polls flag[i] until it is >= value (all lanes), with
// a sleep between polls; past `timeout` wall-clock ticks it sets *err = 1
// and returns, leaving the stream's later work to run on stale data (the
// host checks err after its synchronise and raises).
__global__ __launch_bounds__(64) void wait_flags_kernel(WaitArgs a, int32_t n, int32_t value,
                                                        int32_t *err, uint64_t timeout) {
    const int lane = threadIdx.x;
    const uint64_t t0 = wall_clock64();
    for (;;) {
        bool ok = true;
        if (lane < n)
            ok = __hip_atomic_load(a.flag[lane], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) >=
                 value;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) return;
        if (wall_clock64() - t0 > timeout) {
            if (lane == 0)
                __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

// *flag = value, after everything this stream wrote before it is visible at
// system scope (release store from one lane).
// (The bytes it publishes were stored by earlier kernels of the stream, so
// the kernel boundary's release already wrote them back; the fence covers
// this XCD's L2 again, and the explicit wait keeps the flag store behind the
// write-back: hipcc may drop that wait after buffer_wbl2, MI355X_MICROARCH.md
// "Compiler hazard".)
__global__ __launch_bounds__(64) void signal_flag_kernel(int32_t *flag, int32_t value) {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

int launch_pull_blocks(int32_t nseg, const int64_t *segs, float *dst, int64_t ldd,
                       hipStream_t stream) {
    SGC_REQUIRE(nseg >= 0 && nseg <= kMaxPullSegs, SGC_EINVAL,
                "pull_blocks: %d segments (at most %d)", (int)nseg, kMaxPullSegs);
    SGC_REQUIRE(nseg == 0 || (dst && segs), SGC_EINVAL, "pull_blocks: null pointer");
    SGC_REQUIRE(ldd >= 0, SGC_EINVAL, "pull_blocks: negative stride");
    PullArgs a{};
    int n = 0, V = 4;
    int64_t max_elems = 0;
    for (int s = 0; s < nseg; ++s) {
        // src pointer, src ld, dst_row, dst_col, rows, cols
        const int64_t *q = segs + 6 * s;
        SGC_REQUIRE(q[1] >= 0 && q[2] >= 0 && q[3] >= 0 && q[4] >= 0 && q[5] >= 0, SGC_EINVAL,
                    "pull_blocks: bad segment %d", s);
        if (q[4] == 0 || q[5] == 0) continue;
        SGC_REQUIRE(q[0] != 0 && q[5] <= q[1] && q[3] + q[5] <= ldd, SGC_EINVAL,
                    "pull_blocks: segment %d: null source or columns past a row stride", s);
        SGC_REQUIRE(((q[4] - 1) * q[1] + q[5]) * 4 < ((int64_t)1 << 31), SGC_EINVAL,
                    "pull_blocks: segment %d spans 2 GiB or more (split its rows)", s);
        a.seg[n] = PullSeg{reinterpret_cast<const float *>(q[0]), q[1], q[2] * ldd + q[3],
                           (int32_t)q[4], (int32_t)q[5]};
        for (int64_t x : {q[0] / 4, q[1], q[3], q[5]})
            while (V > 1 && x % V) V >>= 1;
        max_elems = std::max(max_elems, q[4] * q[5]);
        ++n;
    }
    if (n == 0) return SGC_OK;
    while (V > 1 && (ldd % V || reinterpret_cast<uintptr_t>(dst) % (4 * V))) V >>= 1;
    const int64_t per_block = 256LL * kCopyU * V;
    const int64_t blocks = std::max<int64_t>(
        1, std::min<int64_t>((max_elems + per_block - 1) / per_block, 8192 / n + 1));
    const dim3 grid((unsigned)blocks, (unsigned)n);
    if (V == 4)
        hipLaunchKernelGGL((pull_blocks_kernel<4>), grid, dim3(256), 0, stream, dst, ldd, a);
    else if (V == 2)
        hipLaunchKernelGGL((pull_blocks_kernel<2>), grid, dim3(256), 0, stream, dst, ldd, a);
    else
        hipLaunchKernelGGL((pull_blocks_kernel<1>), grid, dim3(256), 0, stream, dst, ldd, a);
    const hipError_t e = hipGetLastError();
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "pull_blocks launch failed: %s", hipGetErrorString(e));
    return SGC_OK;
}

int launch_wait_flags(int32_t n, const int64_t *flags, int32_t value, int32_t *err,
                      int64_t timeout_us, hipStream_t stream) {
    SGC_REQUIRE(n >= 0 && n <= kMaxWaitFlags, SGC_EINVAL, "wait_flags: %d flags (at most %d)",
                (int)n, kMaxWaitFlags);
    SGC_REQUIRE(err && (n == 0 || flags) && timeout_us > 0, SGC_EINVAL,
                "wait_flags: null pointer or timeout <= 0");
    if (n == 0) return SGC_OK;
    WaitArgs a{};
    for (int i = 0; i < n; ++i) {
        SGC_REQUIRE(flags[i] != 0 && flags[i] % 4 == 0, SGC_EINVAL, "wait_flags: bad flag %d", i);
        a.flag[i] = reinterpret_cast<const int32_t *>(flags[i]);
    }
    int dev = 0, khz = 0;
    SGC_HIP_CHECK(hipGetDevice(&dev));
    SGC_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    SGC_REQUIRE(khz > 0, SGC_EHIP, "wait_flags: no wall clock rate");
    const uint64_t ticks = (uint64_t)timeout_us * (uint64_t)khz / 1000;
    hipLaunchKernelGGL(wait_flags_kernel, dim3(1), dim3(kWave), 0, stream, a, n, value, err,
                       ticks);
    const hipError_t e = hipGetLastError();
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "wait_flags launch failed: %s", hipGetErrorString(e));
    return SGC_OK;
}

int launch_signal_flag(int32_t *flag, int32_t value, hipStream_t stream) {
    SGC_REQUIRE(flag && reinterpret_cast<uintptr_t>(flag) % 4 == 0, SGC_EINVAL,
                "signal_flag: bad flag pointer");
    hipLaunchKernelGGL(signal_flag_kernel, dim3(1), dim3(kWave), 0, stream, flag, value);
    const hipError_t e = hipGetLastError();
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "signal_flag launch failed: %s", hipGetErrorString(e));
    return SGC_OK;
}

// The handle of the allocation holding ptr, plus ptr's offset in it (the
// caching allocator hands out pieces of larger allocations): a peer opens
// the allocation and adds the offset.
int ipc_get_handle(const void *ptr, void *handle) {
    SGC_REQUIRE(ptr && handle, SGC_EINVAL, "ipc_get_handle: null pointer");
    static_assert(sizeof(hipIpcMemHandle_t) + sizeof(int64_t) <= SGC_IPC_HANDLE_BYTES,
                  "IPC handle size");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    SGC_HIP_CHECK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)const_cast<void *>(ptr)));
    const int64_t off = (int64_t)(reinterpret_cast<uintptr_t>(ptr) - reinterpret_cast<uintptr_t>(base));
    SGC_REQUIRE(off >= 0 && (size_t)off < size, SGC_EHIP, "ipc_get_handle: pointer outside its range");
    hipIpcMemHandle_t h;
    SGC_HIP_CHECK(hipIpcGetMemHandle(&h, base));
    memset(handle, 0, SGC_IPC_HANDLE_BYTES);
    memcpy(handle, &h, sizeof(h));
    memcpy(static_cast<char *>(handle) + sizeof(h), &off, sizeof(off));
    return SGC_OK;
}

// Opens a peer's handle (ipc_get_handle); *base is what ipc_close takes,
// *ptr the peer's pointer in this process.
int ipc_open(const void *handle, void **base, void **ptr) {
    SGC_REQUIRE(handle && base && ptr, SGC_EINVAL, "ipc_open: null pointer");
    hipIpcMemHandle_t h;
    int64_t off = 0;
    memcpy(&h, handle, sizeof(h));
    memcpy(&off, static_cast<const char *>(handle) + sizeof(h), sizeof(off));
    SGC_REQUIRE(off >= 0, SGC_EINVAL, "ipc_open: bad offset");
    SGC_HIP_CHECK(hipIpcOpenMemHandle(base, h, hipIpcMemLazyEnablePeerAccess));
    *ptr = static_cast<char *>(*base) + off;
    return SGC_OK;
}

int ipc_close(void *base) {
    SGC_REQUIRE(base, SGC_EINVAL, "ipc_close: null pointer");
    SGC_HIP_CHECK(hipIpcCloseMemHandle(base));
    return SGC_OK;
}

int launch_copy_blocks(const float *src, int64_t lds, float *dst, int64_t ldd, int32_t nseg,
                       const int64_t *segs, hipStream_t stream) {
    SGC_REQUIRE(nseg >= 0 && nseg <= kMaxBlockSegs, SGC_EINVAL,
                "copy_blocks: %d segments (at most %d)", (int)nseg, kMaxBlockSegs);
    SGC_REQUIRE(nseg == 0 || (src && dst && segs), SGC_EINVAL, "copy_blocks: null pointer");
    SGC_REQUIRE(lds >= 0 && ldd >= 0, SGC_EINVAL, "copy_blocks: negative stride");
    CopyArgs a{};
    int n = 0, V = 4;
    int64_t max_elems = 0;
    for (int s = 0; s < nseg; ++s) {
        const int64_t *q = segs + 6 * s;  // src_row, src_col, dst_row, dst_col, rows, cols
        SGC_REQUIRE(q[0] >= 0 && q[1] >= 0 && q[2] >= 0 && q[3] >= 0 && q[4] >= 0 && q[5] >= 0 &&
                        q[4] < INT32_MAX && q[5] < INT32_MAX,
                    SGC_EINVAL, "copy_blocks: bad segment %d", s);
        SGC_REQUIRE(q[5] == 0 || (q[1] + q[5] <= lds && q[3] + q[5] <= ldd), SGC_EINVAL,
                    "copy_blocks: segment %d columns past the row stride", s);
        if (q[4] == 0 || q[5] == 0) continue;
        // the flat index runs in 32 bits
        SGC_REQUIRE(q[4] * q[5] < (int64_t)1 << 31, SGC_EINVAL,
                    "copy_blocks: segment %d has %lld elements (at most 2^31 - 1)", s,
                    (long long)(q[4] * q[5]));
        a.seg[n] = CopySeg{q[0] * lds + q[1], q[2] * ldd + q[3], (int32_t)q[4], (int32_t)q[5]};
        for (int64_t x : {q[1], q[3], q[5]})
            while (V > 1 && x % V) V >>= 1;
        max_elems = std::max(max_elems, q[4] * q[5]);
        ++n;
    }
    if (n == 0) return SGC_OK;
    while (V > 1 && (lds % V || ldd % V || reinterpret_cast<uintptr_t>(src) % (4 * V) ||
                     reinterpret_cast<uintptr_t>(dst) % (4 * V)))
        V >>= 1;
    // enough workgroups that each lane copies ~kCopyU vectors of the largest
    // segment, at most ~8k in all (a grid-stride loop covers the rest)
    const int64_t per_block = 256LL * kCopyU * V;
    const int64_t blocks = std::max<int64_t>(
        1, std::min<int64_t>((max_elems + per_block - 1) / per_block, 8192 / n + 1));
    const dim3 grid((unsigned)blocks, (unsigned)n);
    if (V == 4)
        hipLaunchKernelGGL((copy_blocks_kernel<4>), grid, dim3(256), 0, stream, src, lds, dst, ldd, a);
    else if (V == 2)
        hipLaunchKernelGGL((copy_blocks_kernel<2>), grid, dim3(256), 0, stream, src, lds, dst, ldd, a);
    else
        hipLaunchKernelGGL((copy_blocks_kernel<1>), grid, dim3(256), 0, stream, src, lds, dst, ldd, a);
    const hipError_t e = hipGetLastError();
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "copy_blocks launch failed: %s", hipGetErrorString(e));
    return SGC_OK;
}

SGC_WARM_UNIT(warm_exchange)

}  // namespace sgc
