// sort.hip -- the library's own stable LSD radix sort of (key, value) pairs.
//
// Used by the launch plan (rows by degree, longest first: plan.hip) and by
// the ingest of row-unsorted COO input (ingest.hip).  It replaces hipCUB's
// DeviceRadixSort there: the code object of a translation unit is loaded on
// the first launch of any of its kernels, and hipCUB's sort made plan.hip's
// and ingest.hip's 2.2 MB each -- 12-46 ms and 8 ms on the first
// sgc_precompute of a process (profiles/r03/s13/first_call_stages.log) for
// a sort that takes 0.1-0.3 ms.
//
// One pass per 11-bit digit (2,048 bins), each a stable counting sort:
//   count    one 256-thread block per tile of 2,048 pairs: the tile's digit
//            histogram (LDS atomics) -> counts[digit][tile] (digit-major);
//   scan     exclusive scan of counts in that order: the first output slot
//            of every (digit, tile);
//   scatter  the same tiles; each wave takes 512 consecutive pairs of its
//            tile, wave bases per digit from an LDS prefix over the tile's
//            four waves, then 64 pairs at a time: the lanes sharing a digit
//            are found one digit at a time (ballot), ranked by lane order,
//            and the digit's LDS counter advanced -- so equal digits keep
//            their input order and the pass is stable.
// Deterministic: no result depends on atomic order (the count's atomics only
// add).  Descending order compares key_max - key.
#include "sort.h"

#include <algorithm>

namespace sgc {

namespace {

constexpr int kDigitBits = 11;
constexpr int kBins = 1 << kDigitBits;
constexpr int kSortWaves = 4;
constexpr int kPerWave = 512;
constexpr int kTile = kSortWaves * kPerWave;  // pairs per count / scatter block
constexpr int kScanThreads = 256;
constexpr int kScanPer = 16;
constexpr int kScanChunk = kScanThreads * kScanPer;  // entries per scan block

__device__ __forceinline__ uint32_t digit_of(uint32_t key, uint32_t key_max, int desc, int shift) {
    const uint32_t k = desc ? key_max - key : key;
    return (k >> shift) & (kBins - 1);
}

__global__ __launch_bounds__(256) void radix_count_kernel(const uint32_t *__restrict__ keys,
                                                          int64_t n, uint32_t key_max, int desc,
                                                          int shift, int64_t n_tiles,
                                                          uint32_t *__restrict__ counts) {
    __shared__ uint32_t hist[kBins];
    for (int b = threadIdx.x; b < kBins; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kTile;
    for (int i = threadIdx.x; i < kTile; i += blockDim.x) {
        const int64_t k = t0 + i;
        if (k < n) atomicAdd(&hist[digit_of(keys[k], key_max, desc, shift)], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kBins; b += blockDim.x)
        counts[(int64_t)b * n_tiles + blockIdx.x] = hist[b];
}

// Exclusive scan of one value per thread over a block of NT threads; `total`
// gets the block's sum.  wsum: NT / 64 words of LDS.
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *wsum,
                                                         uint32_t &total) {
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
    }
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < NT / kWave; ++i) {
        const uint32_t s = wsum[i];
        if (i < w) before += s;
        total += s;
    }
    __syncthreads();  // wsum may be reused by the caller
    return before + inc - v;
}

__global__ __launch_bounds__(kScanThreads) void scan_blocks_kernel(uint32_t *__restrict__ a,
                                                                   int64_t m,
                                                                   uint32_t *__restrict__ sums) {
    __shared__ uint32_t wsum[kScanThreads / kWave];
    const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanPer;
    uint32_t v[kScanPer];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        v[i] = base + i < m ? a[base + i] : 0u;
        s += v[i];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan<kScanThreads>(s, wsum, total);
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        if (base + i < m) a[base + i] = run;
        run += v[i];
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// One block: exclusive scan of the nb block sums in place.
__global__ __launch_bounds__(1024) void scan_sums_kernel(uint32_t *__restrict__ sums, int64_t nb) {
    __shared__ uint32_t wsum[1024 / kWave];
    uint32_t carry = 0;
    for (int64_t c0 = 0; c0 < nb; c0 += 1024) {
        const int64_t i = c0 + threadIdx.x;
        const uint32_t v = i < nb ? sums[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan<1024>(v, wsum, total);
        if (i < nb) sums[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(kScanThreads) void scan_add_kernel(uint32_t *__restrict__ a, int64_t m,
                                                                const uint32_t *__restrict__ sums) {
    const uint32_t add = sums[blockIdx.x];
    const int64_t base = (int64_t)blockIdx.x * kScanChunk;
    for (int i = threadIdx.x; i < kScanChunk; i += kScanThreads)
        if (base + i < m) a[base + i] += add;
}

__global__ __launch_bounds__(256) void radix_scatter_kernel(
    const uint32_t *__restrict__ keys_in, const int32_t *__restrict__ vals_in,
    uint32_t *__restrict__ keys_out, int32_t *__restrict__ vals_out, int64_t n, uint32_t key_max,
    int desc, int shift, int64_t n_tiles, const uint32_t *__restrict__ offsets) {
    __shared__ uint32_t base[kSortWaves][kBins];  // 32 KB: per-wave next slot of each digit
    const int w = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
    const int64_t w0 = (int64_t)blockIdx.x * kTile + (int64_t)w * kPerWave;
    for (int b = threadIdx.x; b < kSortWaves * kBins; b += blockDim.x) (&base[0][0])[b] = 0;
    __syncthreads();
    for (int i = lane; i < kPerWave; i += kWave) {
        const int64_t k = w0 + i;
        if (k < n) atomicAdd(&base[w][digit_of(keys_in[k], key_max, desc, shift)], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kBins; b += blockDim.x) {  // waves of the tile in order
        uint32_t run = offsets[(int64_t)b * n_tiles + blockIdx.x];
#pragma unroll
        for (int i = 0; i < kSortWaves; ++i) {
            const uint32_t c = base[i][b];
            base[i][b] = run;
            run += c;
        }
    }
    __syncthreads();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (kWave - lane));  // lanes below this one
    for (int c0 = 0; c0 < kPerWave; c0 += kWave) {
        const int64_t k = w0 + c0 + lane;
        const bool valid = k < n;
        const uint32_t key = valid ? keys_in[k] : 0u;
        const int32_t val = valid ? vals_in[k] : 0;
        const uint32_t d = valid ? digit_of(key, key_max, desc, shift) : 0xffffffffu;
        uint64_t todo = __ballot(valid);
        uint32_t pos = 0;
        while (todo) {  // wave-uniform: one digit present in this chunk per iteration
            const int lead = __builtin_ctzll(todo);
            const uint32_t dl = (uint32_t)__builtin_amdgcn_readlane((int)d, lead);
            const uint64_t same = __ballot(d == dl);
            if (d == dl) pos = base[w][dl] + (uint32_t)__popcll(same & lt);
            if (lane == lead) base[w][dl] += (uint32_t)__popcll(same);
            todo &= ~same;
        }
        if (valid) {
            keys_out[pos] = key;
            vals_out[pos] = val;
        }
    }
}

struct SortLayout {
    int64_t n_tiles, m, n_scan;
    uint32_t *counts, *sums, *keys_tmp;
    int32_t *vals_tmp;
    size_t bytes;
};

SortLayout layout(int64_t n, char *base) {
    SortLayout L{};
    L.n_tiles = (n + kTile - 1) / kTile;
    L.m = L.n_tiles * kBins;
    L.n_scan = (L.m + kScanChunk - 1) / kScanChunk;
    size_t used = 0;
    auto take = [&](size_t bytes) {
        used = (used + 255) & ~size_t(255);
        char *p = base ? base + used : nullptr;
        used += bytes;
        return p;
    };
    L.counts = reinterpret_cast<uint32_t *>(take((size_t)L.m * 4));
    L.sums = reinterpret_cast<uint32_t *>(take((size_t)std::max<int64_t>(1, L.n_scan) * 4));
    L.keys_tmp = reinterpret_cast<uint32_t *>(take((size_t)n * 4));
    L.vals_tmp = reinterpret_cast<int32_t *>(take((size_t)n * 4));
    L.bytes = used + 256;
    return L;
}

}  // namespace

int64_t radix_sort_workspace(int64_t n) { return (int64_t)layout(std::max<int64_t>(n, 0), nullptr).bytes; }

int radix_sort_pairs(const uint32_t *keys_in, const int32_t *vals_in, uint32_t *keys_out,
                     int32_t *vals_out, int64_t n, uint32_t key_max, bool descending, void *ws,
                     int64_t ws_bytes, hipStream_t stream) {
    SGC_REQUIRE(n >= 0 && n < INT32_MAX, SGC_ERANGE, "radix_sort: bad size %lld", (long long)n);
    if (n == 0) return SGC_OK;
    SGC_REQUIRE(keys_in && vals_in && keys_out && vals_out && ws, SGC_EINVAL,
                "radix_sort: null pointer");
    const SortLayout L = layout(n, static_cast<char *>(ws));
    SGC_REQUIRE(ws_bytes >= (int64_t)L.bytes, SGC_ENOMEM, "radix_sort: workspace %lld < %zu",
                (long long)ws_bytes, L.bytes);
    int bits = 0;
    while (bits < 32 && (key_max >> bits) != 0) ++bits;
    const int passes = std::max(1, (bits + kDigitBits - 1) / kDigitBits);
    const uint32_t *ks = keys_in;
    const int32_t *vs = vals_in;
    for (int p = 0; p < passes; ++p) {
        // the last pass writes the output; the ones before alternate so that
        // no pass reads the buffer it writes
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        uint32_t *kd = to_out ? keys_out : L.keys_tmp;
        int32_t *vd = to_out ? vals_out : L.vals_tmp;
        const int shift = p * kDigitBits;
        hipLaunchKernelGGL(radix_count_kernel, dim3((unsigned)L.n_tiles), dim3(256), 0, stream, ks,
                           n, key_max, (int)descending, shift, L.n_tiles, L.counts);
        SGC_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(scan_blocks_kernel, dim3((unsigned)L.n_scan), dim3(kScanThreads), 0,
                           stream, L.counts, L.m, L.sums);
        SGC_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(1024), 0, stream, L.sums, L.n_scan);
        SGC_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(scan_add_kernel, dim3((unsigned)L.n_scan), dim3(kScanThreads), 0, stream,
                           L.counts, L.m, L.sums);
        SGC_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(radix_scatter_kernel, dim3((unsigned)L.n_tiles), dim3(256), 0, stream,
                           ks, vs, kd, vd, n, key_max, (int)descending, shift, L.n_tiles, L.counts);
        SGC_HIP_CHECK(hipGetLastError());
        ks = kd;
        vs = vd;
    }
    return SGC_OK;
}

SGC_WARM_UNIT(warm_sort)

}  // namespace sgc
