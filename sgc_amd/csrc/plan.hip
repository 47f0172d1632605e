// plan.hip -- the launch plan on the device: every row of [row_begin,
// row_end) sorted by degree, longest first, ties in row order (one stable
// radix sort), plus the counts the launch geometry needs -- rows above the
// heavy threshold, above the hub threshold, and the longest row -- read back
// in ONE small copy.  The sorted list is exactly what sgc_plan_build +
// sgc_plan_light_order produce together (heavy rows heaviest first, then the
// light rows longest first; SGC_SPMM_LIGHT_ORDER), without their host sorts,
// their row_ptr read-back and three of their four synchronisations.
// A schedule only: results never depend on it.
// The sort is the library's own (sort.hip, 11-bit digits: two passes up to
// degree 4,194,303): hipCUB's made this translation unit's code object
// 2.2 MB, whose load cost the first plan of a process 12-46 ms.
#include "common.h"
#include "sort.h"

namespace sgc {

namespace {

__global__ void plan_keys_kernel(const int32_t *__restrict__ row_ptr, int row_begin, int n_rows,
                                 int threshold, int hub_threshold, uint32_t *__restrict__ deg,
                                 int32_t *__restrict__ ids, int32_t *__restrict__ counts) {
    int heavy = 0, hub = 0, top = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_rows;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int row = row_begin + (int)i;
        const int d = row_ptr[row + 1] - row_ptr[row];
        deg[i] = (uint32_t)d;
        ids[i] = row;
        heavy += d > threshold;
        hub += d > hub_threshold;
        top = max(top, d);
    }
    // wave-level reduction, then one atomic per wave (vector atomics)
    for (int o = 32; o > 0; o >>= 1) {
        heavy += __shfl_xor(heavy, o);
        hub += __shfl_xor(hub, o);
        top = max(top, __shfl_xor(top, o));
    }
    if ((threadIdx.x & (kWave - 1)) == 0) {
        if (heavy) atomicAdd(&counts[0], heavy);
        if (hub) atomicAdd(&counts[1], hub);
        atomicMax(&counts[2], top);
    }
}

size_t sort_temp_bytes(int64_t n) { return (size_t)radix_sort_workspace(n); }

constexpr size_t kAlign = 256;
size_t up(size_t b) { return (b + kAlign - 1) / kAlign * kAlign; }

}  // namespace

int64_t plan_sorted_workspace(int64_t n_rows) {
    if (n_rows <= 0) return (int64_t)kAlign;
    return (int64_t)(up(3 * sizeof(int32_t)) + 3 * up((size_t)n_rows * sizeof(int32_t)) +
                     up(sort_temp_bytes(n_rows)));
}

int plan_sorted(const int32_t *row_ptr, int64_t row_begin, int64_t row_end, int32_t threshold,
                int32_t hub_threshold, int32_t *plan, void *workspace, int64_t workspace_bytes,
                int64_t *counts_host, hipStream_t stream) {
    SGC_REQUIRE(row_ptr && plan && counts_host && workspace, SGC_EINVAL, "plan_sorted: null pointer");
    SGC_REQUIRE(hub_threshold >= threshold && threshold >= 0, SGC_EINVAL,
                "plan_sorted: need 0 <= threshold <= hub_threshold");
    const int64_t n = row_end - row_begin;
    SGC_REQUIRE(n >= 0 && row_begin >= 0 && row_end < INT32_MAX, SGC_ERANGE,
                "plan_sorted: bad row range");
    counts_host[0] = counts_host[1] = counts_host[2] = 0;
    if (n == 0) return SGC_OK;
    SGC_REQUIRE(workspace_bytes >= plan_sorted_workspace(n), SGC_ENOMEM,
                "plan_sorted: workspace %lld < %lld bytes", (long long)workspace_bytes,
                (long long)plan_sorted_workspace(n));
    char *w = static_cast<char *>(workspace);
    int32_t *counts = reinterpret_cast<int32_t *>(w);
    w += up(3 * sizeof(int32_t));
    uint32_t *deg = reinterpret_cast<uint32_t *>(w);
    w += up((size_t)n * sizeof(int32_t));
    uint32_t *deg_sorted = reinterpret_cast<uint32_t *>(w);
    w += up((size_t)n * sizeof(int32_t));
    int32_t *ids = reinterpret_cast<int32_t *>(w);
    w += up((size_t)n * sizeof(int32_t));
    size_t temp = sort_temp_bytes(n);
    SGC_HIP_CHECK(hipMemsetAsync(counts, 0, 3 * sizeof(int32_t), stream));
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(plan_keys_kernel, dim3(blocks), dim3(256), 0, stream, row_ptr,
                       (int)row_begin, (int)n, threshold, hub_threshold, deg, ids, counts);
    SGC_HIP_CHECK(hipGetLastError());
    int32_t c[3] = {0, 0, 0};
    SGC_HIP_CHECK(hipMemcpyAsync(c, counts, sizeof(c), hipMemcpyDeviceToHost, stream));
    SGC_HIP_CHECK(hipStreamSynchronize(stream));
    counts_host[0] = c[0];
    counts_host[1] = c[1];
    counts_host[2] = c[2];
    // stable: equal degrees keep ascending row order; the longest row (read
    // back above) sets the passes.  Waited for, so the plan (and the
    // workspace) may be used from any stream once this returns.
    const int rc = radix_sort_pairs(deg, ids, deg_sorted, plan, n, (uint32_t)std::max(0, c[2]),
                                    true, w, (int64_t)temp, stream);
    if (rc != SGC_OK) return rc;
    SGC_HIP_CHECK(hipStreamSynchronize(stream));
    return SGC_OK;
}

SGC_WARM_UNIT(warm_plan)

}  // namespace sgc
