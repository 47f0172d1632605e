// capi.hip -- extern "C" entry points of libsgc_amd.so (include/sgc_amd.h).
#include <cstdarg>
#include <map>
#include <mutex>
#include <vector>
#include <cstdio>

#include "common.h"

namespace sgc {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int coo_to_csr_workspace(int64_t n_rows, int64_t nnz, size_t *bytes);
int coo_to_csr(const int64_t *rows, const int64_t *cols, const float *vals, int64_t nnz,
               int64_t n_rows, int64_t n_cols, int32_t *row_ptr, int32_t *col_idx,
               float *val_out, void *ws, size_t ws_bytes, uint32_t *status_host,
               hipStream_t stream);
int csr64_to_csr(const int64_t *crow, const int64_t *col, const float *vals, int64_t nnz,
                 int64_t n_rows, int64_t n_cols, int32_t *row_ptr, int32_t *col_idx,
                 float *val_out, uint32_t *status_host, hipStream_t stream);
int build_plan(const int32_t *row_ptr, int64_t row_begin, int64_t row_end, int32_t threshold,
               int32_t hub_threshold, int32_t *plan, int64_t capacity, int64_t *n_heavy_host,
               int64_t *n_hub_host, hipStream_t stream);
int light_order(const int32_t *row_ptr, int64_t row_begin, int64_t row_end, int32_t threshold,
                int32_t *light, int64_t *n_light_host, hipStream_t stream);
int launch_spmm(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                int64_t row_begin, int64_t row_end, const float *X, int64_t ldx, float *Y,
                int64_t ldy, int64_t F, const int32_t *heavy_rows, int64_t n_heavy,
                int64_t n_hub, int32_t heavy_threshold, uint32_t flags, hipStream_t stream);
int launch_pad_rows(const float *src, int64_t lds, float *dst, int64_t ldd, int64_t n_rows,
                    int64_t F, hipStream_t stream);
int launch_copy_blocks(const float *src, int64_t lds, float *dst, int64_t ldd, int32_t nseg,
                       const int64_t *segs, hipStream_t stream);
int launch_pull_blocks(int32_t nseg, const int64_t *segs, float *dst, int64_t ldd,
                       hipStream_t stream);
int launch_wait_flags(int32_t n, const int64_t *flags, int32_t value, int32_t *err,
                      int64_t timeout_us, hipStream_t stream);
int launch_signal_flag(int32_t *flag, int32_t value, hipStream_t stream);
int ipc_get_handle(const void *ptr, void *handle);
int ipc_open(const void *handle, void **base, void **ptr);
int ipc_close(void *base);
size_t augnorm_scan_temp_bytes(int64_t n);
int augnorm_count(const int32_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                  int64_t nnz, int32_t *out_row_ptr, double *rowsum, void *ws, size_t ws_bytes,
                  int64_t *out_nnz_host, uint32_t *status_host, hipStream_t s);
int augnorm_fill(const int32_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                 const double *d, int32_t *out_row_ptr, int32_t *out_col, float *out_val,
                 void *ws, size_t ws_bytes, int64_t *out_nnz_host, hipStream_t s);
int csr_to_coo64(const int32_t *row_ptr, const int32_t *col, int64_t n, int64_t *rows64,
                 int64_t *cols64, hipStream_t s);
int64_t xent_workspace_bytes(int64_t M, int64_t K, int64_t C);
int linear_xent_f32(const float *X, int64_t ldx, const float *W, const float *b,
                    const int64_t *labels, int64_t M, int64_t K, int64_t C, float *loss,
                    float *dW, float *db, float *logits, int64_t ldl, void *ws, int64_t ws_bytes,
                    hipStream_t s);
int64_t cross_entropy_workspace(int64_t M, int64_t C);
int cross_entropy_fwd_f32(const float *Y, int64_t ldy, const int64_t *labels, int64_t M, int64_t C,
                          int64_t ignore_index, float *loss, float *inv_count, float *lse, void *ws,
                          int64_t ws_bytes, hipStream_t s);
int cross_entropy_bwd_f32(const float *Y, int64_t ldy, const int64_t *labels, const float *lse,
                          const float *inv_count, const float *grad, int64_t M, int64_t C,
                          int64_t ignore_index, float *dY, int64_t lddy, hipStream_t s);
int64_t linear_backward_workspace_bytes(int64_t M, int64_t K, int64_t C);
int linear_backward_f32(const float *X, int64_t ldx, const float *dY, int64_t ldd, int64_t M,
                        int64_t K, int64_t C, float *dW, float *db, void *ws, int64_t ws_bytes,
                        hipStream_t s);
int64_t subgraph_workspace(int64_t n, int64_t m, int64_t nnz);
int subgraph_count(const int32_t *row_ptr, const int32_t *col, int64_t n, const int64_t *idx,
                   int64_t m, int64_t nnz, int32_t *out_row_ptr, void *ws, int64_t ws_bytes,
                   int64_t *out_nnz_host, uint32_t *status_host, hipStream_t s);
int subgraph_fill(const int32_t *row_ptr, const int32_t *col, const double *val, int64_t n,
                  const int64_t *idx, int64_t m, int64_t nnz, const int32_t *out_row_ptr,
                  int32_t *out_col, double *out_val, void *ws, int64_t ws_bytes, hipStream_t s);
int set_tuning(const char *key, int64_t value);
int64_t get_tuning(const char *key);
int timing_enable(int on);
int timing_collect(float *light_ms, float *hub_ms, int64_t capacity, int64_t *n_host);
int timing_collect_ex(float *light_ms, float *hub_ms, float *span_ms, int32_t *kernel,
                      int64_t capacity, int64_t *n_host);
int coo_to_csr_cpu(const int64_t *rows, const int64_t *cols, const float *vals, int64_t nnz,
                   int64_t n_rows, int64_t n_cols, int32_t *row_ptr, int32_t *col_idx,
                   float *val_out, uint32_t *status_host);
int spmm_cpu(const int32_t *row_ptr, const int32_t *col_idx, const float *val, int64_t row_begin,
             int64_t row_end, const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
             int32_t n_threads, bool accum);
int64_t propagate_cpu_workspace(int64_t n_rows, int64_t F, int32_t K);
int propagate_cpu(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                  int64_t n_rows, const float *X0, int64_t ldx, float *out, int64_t ldo, int64_t F,
                  int32_t K, void *workspace, int64_t workspace_bytes, int32_t n_threads);
const char *linear_kernel_name(int64_t M, int64_t K, int64_t ldx, int64_t C, const float *X);
const char *linear_backward_kernel_name(int64_t M, int64_t K, int64_t ldx, int64_t C,
                                        const float *X);
int launch_linear_f32(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                      int64_t ldy, int64_t M, int64_t K, int64_t C, hipStream_t stream);
int64_t plan_sorted_workspace(int64_t n_rows);
int plan_sorted(const int32_t *row_ptr, int64_t row_begin, int64_t row_end, int32_t threshold,
                int32_t hub_threshold, int32_t *plan, void *workspace, int64_t workspace_bytes,
                int64_t *counts_host, hipStream_t stream);
int64_t colsplit_workspace(int64_t n_rows, int32_t groups);
int colsplit(const int32_t *row_ptr, const int32_t *col_idx, const float *val, int64_t n_rows,
             int64_t n_cols, int32_t groups, const int32_t *cuts_host, int32_t *row_ptrs,
             int32_t *col_out, float *val_out, void *workspace, int64_t workspace_bytes,
             hipStream_t stream);
int mgpu_init(int ndev, const int *devices);
int mgpu_finalize();
int mgpu_attach(const int32_t *row_ptr, const int32_t *col_idx, const float *val, int64_t n,
                int64_t nnz, hipStream_t stream, int64_t *handle);
int mgpu_detach(int64_t handle);
int mgpu_propagate(int64_t handle, const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                   int32_t K, hipStream_t stream);

}  // namespace sgc

using namespace sgc;

extern "C" {

int sgc_abi_version(void) { return SGC_ABI_VERSION; }

const char *sgc_last_error(void) { return g_err; }

int sgc_set_tuning(const char *key, int64_t value) { return set_tuning(key, value); }

int64_t sgc_get_tuning(const char *key) { return get_tuning(key); }

int sgc_coo_to_csr_workspace(int64_t n_rows, int64_t nnz, size_t *bytes_host) {
    return coo_to_csr_workspace(n_rows, nnz, bytes_host);
}

int sgc_coo_to_csr(const int64_t *rows, const int64_t *cols, const float *vals, int64_t nnz,
                   int64_t n_rows, int64_t n_cols, int32_t *row_ptr, int32_t *col_idx,
                   float *val_out, void *workspace, size_t workspace_bytes,
                   uint32_t *status_host, void *stream) {
    return coo_to_csr(rows, cols, vals, nnz, n_rows, n_cols, row_ptr, col_idx, val_out, workspace,
                      workspace_bytes, status_host, as_stream(stream));
}

int sgc_csr64_to_csr(const int64_t *crow, const int64_t *col, const float *vals, int64_t nnz,
                     int64_t n_rows, int64_t n_cols, int32_t *row_ptr, int32_t *col_idx,
                     float *val_out, uint32_t *status_host, void *stream) {
    return csr64_to_csr(crow, col, vals, nnz, n_rows, n_cols, row_ptr, col_idx, val_out,
                        status_host, as_stream(stream));
}

int64_t sgc_augnorm_workspace(int64_t n_rows) {
    const int64_t n = n_rows < 1 ? 1 : n_rows;
    return 4 * ((n * 4 + 255) / 256 * 256) + (int64_t)augnorm_scan_temp_bytes(n) + 1024;
}

int sgc_augnorm_count(const int32_t *row_ptr, const int32_t *col_idx, const double *val,
                      int64_t n_rows, int64_t nnz, int32_t *out_row_ptr, double *rowsum,
                      void *workspace, int64_t workspace_bytes, int64_t *out_nnz_host,
                      uint32_t *status_host, void *stream) {
    SGC_REQUIRE(out_nnz_host, SGC_EINVAL, "augnorm_count: null out_nnz_host");
    return augnorm_count(row_ptr, col_idx, val, n_rows, nnz, out_row_ptr, rowsum, workspace,
                         workspace_bytes < 0 ? 0 : (size_t)workspace_bytes, out_nnz_host,
                         status_host, as_stream(stream));
}

int sgc_augnorm_fill(const int32_t *row_ptr, const int32_t *col_idx, const double *val,
                     int64_t n_rows, const double *d, int32_t *out_row_ptr, int32_t *out_col_idx,
                     float *out_val, void *workspace, int64_t workspace_bytes,
                     int64_t *out_nnz_host, void *stream) {
    SGC_REQUIRE(out_nnz_host, SGC_EINVAL, "augnorm_fill: null out_nnz_host");
    return augnorm_fill(row_ptr, col_idx, val, n_rows, d, out_row_ptr, out_col_idx, out_val,
                        workspace, workspace_bytes < 0 ? 0 : (size_t)workspace_bytes,
                        out_nnz_host, as_stream(stream));
}

int64_t sgc_subgraph_workspace(int64_t n_rows, int64_t m, int64_t nnz) {
    return subgraph_workspace(n_rows, m, nnz);
}

int sgc_subgraph_count(const int32_t *row_ptr, const int32_t *col_idx, int64_t n_rows,
                       int64_t nnz, const int64_t *idx, int64_t m, int32_t *out_row_ptr,
                       void *workspace, int64_t workspace_bytes, int64_t *out_nnz_host,
                       uint32_t *status_host, void *stream) {
    return subgraph_count(row_ptr, col_idx, n_rows, idx, m, nnz, out_row_ptr, workspace,
                          workspace_bytes, out_nnz_host, status_host, as_stream(stream));
}

int sgc_subgraph_fill(const int32_t *row_ptr, const int32_t *col_idx, const double *val,
                      int64_t n_rows, int64_t nnz, const int64_t *idx, int64_t m,
                      const int32_t *out_row_ptr, int32_t *out_col_idx, double *out_val,
                      void *workspace, int64_t workspace_bytes, void *stream) {
    return subgraph_fill(row_ptr, col_idx, val, n_rows, idx, m, nnz, out_row_ptr, out_col_idx,
                         out_val, workspace, workspace_bytes, as_stream(stream));
}

int sgc_csr_to_coo64(const int32_t *row_ptr, const int32_t *col_idx, int64_t n_rows,
                     int64_t *rows64, int64_t *cols64, void *stream) {
    return csr_to_coo64(row_ptr, col_idx, n_rows, rows64, cols64, as_stream(stream));
}

int64_t sgc_plan_capacity(int64_t n_rows) { return 2 * (n_rows < 0 ? 0 : n_rows) + 1; }

int sgc_plan_light_order(const int32_t *row_ptr, int64_t row_begin, int64_t row_end,
                         int32_t heavy_threshold, int32_t *light, int64_t *n_light_host,
                         void *stream) {
    return light_order(row_ptr, row_begin, row_end, heavy_threshold, light, n_light_host,
                       as_stream(stream));
}

int sgc_plan_build(const int32_t *row_ptr, int64_t row_begin, int64_t row_end,
                   int32_t heavy_threshold, int32_t hub_threshold, int32_t *plan,
                   int64_t plan_capacity, int64_t *n_heavy_host, int64_t *n_hub_host,
                   void *stream) {
    return build_plan(row_ptr, row_begin, row_end, heavy_threshold, hub_threshold, plan,
                      plan_capacity, n_heavy_host, n_hub_host, as_stream(stream));
}

int sgc_spmm_csr_f32(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                     int64_t row_begin, int64_t row_end, const float *X, int64_t ldx, float *Y,
                     int64_t ldy, int64_t F, const int32_t *plan, int64_t n_heavy,
                     int64_t n_hub, int32_t heavy_threshold, void *stream) {
    return launch_spmm(row_ptr, col_idx, val, row_begin, row_end, X, ldx, Y, ldy, F, plan,
                       plan ? n_heavy : 0, plan ? n_hub : 0, heavy_threshold, 0u,
                       as_stream(stream));
}

int sgc_spmm_csr_f32_ex(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                        int64_t row_begin, int64_t row_end, const float *X, int64_t ldx, float *Y,
                        int64_t ldy, int64_t F, const int32_t *plan, int64_t n_heavy,
                        int64_t n_hub, int32_t heavy_threshold, uint32_t flags, void *stream) {
    constexpr uint32_t known = SGC_SPMM_X_PADDED | SGC_SPMM_Y_PADDED | SGC_SPMM_NO_HUB |
                               SGC_SPMM_HUB_ONLY | SGC_SPMM_ACCUMULATE | SGC_SPMM_HUB_SERIAL |
                               SGC_SPMM_LIGHT_ORDER | SGC_SPMM_X_UNDER_4G;
    SGC_REQUIRE((flags & ~known) == 0, SGC_EINVAL, "spmm_ex: unknown flags 0x%x", flags);
    SGC_REQUIRE(!((flags & SGC_SPMM_NO_HUB) && (flags & SGC_SPMM_HUB_ONLY)), SGC_EINVAL,
                "spmm_ex: NO_HUB and HUB_ONLY together");
    return launch_spmm(row_ptr, col_idx, val, row_begin, row_end, X, ldx, Y, ldy, F, plan,
                       plan ? n_heavy : 0, plan ? n_hub : 0, heavy_threshold, flags,
                       as_stream(stream));
}

int64_t sgc_aligned_ld(int64_t F) { return F <= 0 ? 0 : (F + 31) / 32 * 32; }

static bool needs_pad(int64_t ldx, const float *X0) {
    return (ldx % 32) != 0 || (reinterpret_cast<uintptr_t>(X0) % 128) != 0;
}

int64_t sgc_propagate_workspace(int64_t n_rows, int64_t F, int64_t ldx, int32_t K) {
    if (n_rows <= 0 || F <= 0 || K <= 0) return 0;
    const int64_t buf = n_rows * sgc_aligned_ld(F) * 4 + 256;
    (void)ldx;  // sized for the padded-input case (the pointer's alignment is unknown here)
    return (K >= 2 ? 2 : 1) * buf + 256;
}

int sgc_pad_rows_f32(const float *src, int64_t lds, float *dst, int64_t ldd, int64_t n_rows,
                     int64_t F, void *stream) {
    return launch_pad_rows(src, lds, dst, ldd, n_rows, F, as_stream(stream));
}

int sgc_copy_blocks_f32(const float *src, int64_t lds, float *dst, int64_t ldd, int32_t nseg,
                        const int64_t *segs_host, void *stream) {
    return launch_copy_blocks(src, lds, dst, ldd, nseg, segs_host, as_stream(stream));
}

int sgc_ipc_get_handle(const void *ptr, void *handle_host) { return ipc_get_handle(ptr, handle_host); }

int sgc_ipc_open(const void *handle_host, void **base_host, void **ptr_host) {
    return ipc_open(handle_host, base_host, ptr_host);
}

int sgc_ipc_close(void *base) { return ipc_close(base); }

int sgc_signal_flag_i32(int32_t *flag, int32_t value, void *stream) {
    return launch_signal_flag(flag, value, as_stream(stream));
}

int sgc_wait_flags_i32(int32_t n, const int64_t *flag_ptrs_host, int32_t value, int32_t *err,
                       int64_t timeout_us, void *stream) {
    return launch_wait_flags(n, flag_ptrs_host, value, err, timeout_us, as_stream(stream));
}

int sgc_pull_blocks_f32(int32_t nseg, const int64_t *segs_host, float *dst, int64_t ldd,
                        void *stream) {
    return launch_pull_blocks(nseg, segs_host, dst, ldd, as_stream(stream));
}

// Recorded launch lists (sgc_launch_list_*): the K-hop loop's launches built
// once with their arguments, replayed by one call per propagation.  X_0 and
// X_K enter by slot, so one list serves every feature tensor of the recorded
// shape / strides / alignment on its stream.
}  // extern "C"

namespace sgc {
namespace {

struct ListOp {
    int kind;  // 0 spmm (launch_spmm), 1 pad rows (launch_pad_rows)
    const int32_t *row_ptr, *col_idx;
    const float *val;
    int64_t row_begin, row_end;
    const float *X;
    int64_t ldx;
    float *Y;
    int64_t ldy, F;
    const int32_t *plan;
    int64_t n_heavy, n_hub;
    int32_t threshold;
    uint32_t flags;
    int32_t x_slot, y_slot;  // SGC_SLOT_*: the pointer as recorded, or the run's X_0 / X_K
};

struct LaunchList {
    int device = 0;
    std::vector<ListOp> ops;
};

std::mutex g_lists_mu;
std::map<int64_t, LaunchList> g_lists;
int64_t g_next_list = 1;

template <typename T>
T *slot_ptr(T *recorded, int32_t slot, const float *X, float *out) {
    if (slot == SGC_SLOT_X0) return (T *)X;
    if (slot == SGC_SLOT_OUT) return (T *)out;
    return recorded;
}

}  // namespace
}  // namespace sgc

extern "C" {

int sgc_launch_list_create(int64_t *handle_host) {
    SGC_REQUIRE(handle_host, SGC_EINVAL, "launch_list_create: null handle");
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "launch_list_create: %s", hipGetErrorString(e));
    std::lock_guard<std::mutex> lock(g_lists_mu);
    const int64_t h = g_next_list++;
    g_lists[h].device = dev;
    *handle_host = h;
    return SGC_OK;
}

int sgc_launch_list_destroy(int64_t handle) {
    std::lock_guard<std::mutex> lock(g_lists_mu);
    SGC_REQUIRE(g_lists.erase(handle) == 1, SGC_EINVAL, "launch_list_destroy: unknown handle %lld",
                (long long)handle);
    return SGC_OK;
}

static int list_add(int64_t handle, const ListOp &op) {
    SGC_REQUIRE(op.x_slot >= SGC_SLOT_FIXED && op.x_slot <= SGC_SLOT_OUT && op.y_slot >= SGC_SLOT_FIXED &&
                    op.y_slot <= SGC_SLOT_OUT,
                SGC_EINVAL, "launch_list_add: bad slot (%d, %d)", op.x_slot, op.y_slot);
    std::lock_guard<std::mutex> lock(g_lists_mu);
    auto it = g_lists.find(handle);
    SGC_REQUIRE(it != g_lists.end(), SGC_EINVAL, "launch_list_add: unknown handle %lld",
                (long long)handle);
    it->second.ops.push_back(op);
    return SGC_OK;
}

int sgc_launch_list_add_spmm(int64_t handle, const int32_t *row_ptr, const int32_t *col_idx,
                             const float *val, int64_t row_begin, int64_t row_end, const float *X,
                             int64_t ldx, float *Y, int64_t ldy, int64_t F, const int32_t *plan,
                             int64_t n_heavy, int64_t n_hub, int32_t heavy_threshold,
                             uint32_t flags, int32_t x_slot, int32_t y_slot) {
    constexpr uint32_t known = SGC_SPMM_X_PADDED | SGC_SPMM_Y_PADDED | SGC_SPMM_NO_HUB |
                               SGC_SPMM_HUB_ONLY | SGC_SPMM_ACCUMULATE | SGC_SPMM_HUB_SERIAL |
                               SGC_SPMM_LIGHT_ORDER | SGC_SPMM_X_UNDER_4G;
    SGC_REQUIRE((flags & ~known) == 0, SGC_EINVAL, "launch_list_add_spmm: unknown flags 0x%x", flags);
    SGC_REQUIRE(!((flags & SGC_SPMM_NO_HUB) && (flags & SGC_SPMM_HUB_ONLY)), SGC_EINVAL,
                "launch_list_add_spmm: NO_HUB and HUB_ONLY together");
    return list_add(handle, ListOp{0, row_ptr, col_idx, val, row_begin, row_end, X, ldx, Y, ldy, F,
                                   plan, plan ? n_heavy : 0, plan ? n_hub : 0, heavy_threshold,
                                   flags, x_slot, y_slot});
}

int sgc_launch_list_add_pad_rows(int64_t handle, const float *src, int64_t lds, float *dst,
                                 int64_t ldd, int64_t n_rows, int64_t F, int32_t src_slot,
                                 int32_t dst_slot) {
    return list_add(handle, ListOp{1, nullptr, nullptr, nullptr, 0, n_rows, src, lds, dst, ldd, F,
                                   nullptr, 0, 0, 0, 0u, src_slot, dst_slot});
}

int sgc_launch_list_run(int64_t handle, const float *X0, float *out, void *stream) {
    // held for the whole run (a few launches): a concurrent destroy of this
    // list from another thread waits instead of freeing it under the run
    std::lock_guard<std::mutex> lock(g_lists_mu);
    auto it = g_lists.find(handle);
    SGC_REQUIRE(it != g_lists.end(), SGC_EINVAL, "launch_list_run: unknown handle %lld",
                (long long)handle);
    const LaunchList *L = &it->second;
    int cur = 0;
    hipError_t e = hipGetDevice(&cur);
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "launch_list_run: %s", hipGetErrorString(e));
    if (cur != L->device) {
        e = hipSetDevice(L->device);
        SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "launch_list_run: %s", hipGetErrorString(e));
    }
    hipStream_t s = as_stream(stream);
    int rc = SGC_OK;
    for (const ListOp &op : L->ops) {
        const float *x = slot_ptr(op.X, op.x_slot, X0, out);
        float *y = slot_ptr(op.Y, op.y_slot, X0, out);
        if (!x || !y) {
            set_error("launch_list_run: null X_0 / X_K for a slot");
            rc = SGC_EINVAL;
            break;
        }
        rc = op.kind == 0 ? launch_spmm(op.row_ptr, op.col_idx, op.val, op.row_begin, op.row_end, x,
                                        op.ldx, y, op.ldy, op.F, op.plan, op.n_heavy, op.n_hub,
                                        op.threshold, op.flags, s)
                          : launch_pad_rows(x, op.ldx, y, op.ldy, op.row_end, op.F, s);
        if (rc != SGC_OK) break;
    }
    if (cur != L->device) (void)hipSetDevice(cur);
    return rc;
}

int sgc_propagate_groups_f32(int32_t groups, const int32_t *row_ptrs, const int32_t *col_idx,
                             const float *val, int64_t n_rows, const float *X0, int64_t ldx,
                             float *out, int64_t ldo, int64_t F, int32_t K,
                             const int32_t *const *plans_host, const int64_t *n_heavy_host,
                             const int64_t *n_hub_host, const int32_t *thresholds_host,
                             const uint32_t *plan_flags_host, void *workspace,
                             int64_t workspace_bytes, void *stream) {
    hipStream_t s = as_stream(stream);
    SGC_REQUIRE(K >= 0, SGC_EINVAL, "propagate: negative degree %d", K);
    SGC_REQUIRE(groups >= 1 && groups <= 8, SGC_EINVAL, "propagate: groups must be 1..8");
    SGC_REQUIRE(X0 && out && row_ptrs, SGC_EINVAL, "propagate: null pointer");
    SGC_REQUIRE(ldx >= F && ldo >= F && F >= 0 && n_rows >= 0, SGC_EINVAL, "propagate: bad shape");
    SGC_REQUIRE(!plans_host || (n_heavy_host && n_hub_host && thresholds_host), SGC_EINVAL,
                "propagate: plans without their counts");
    constexpr uint32_t kPlanFlags = SGC_SPMM_LIGHT_ORDER | SGC_SPMM_HUB_SERIAL;
    if (plan_flags_host)
        for (int g = 0; g < groups; ++g)
            SGC_REQUIRE((plan_flags_host[g] & ~kPlanFlags) == 0, SGC_EINVAL,
                        "propagate: plan flags may only be LIGHT_ORDER / HUB_SERIAL");
    if (K == 0)
        return sgc_pad_rows_f32(X0, ldx, out, ldo, n_rows, F, stream);
    if (n_rows == 0 || F == 0) return SGC_OK;
    const int64_t need = sgc_propagate_workspace(n_rows, F, ldx, K);
    SGC_REQUIRE(workspace_bytes >= need && (need == 0 || workspace), SGC_ENOMEM,
                "propagate: workspace %lld < %lld bytes", (long long)workspace_bytes,
                (long long)need);
    const int64_t ldw = sgc_aligned_ld(F);
    const int64_t buf_floats = (n_rows * ldw * 4 + 256) / 4;
    uintptr_t base = (reinterpret_cast<uintptr_t>(workspace) + 255) & ~uintptr_t(255);
    float *bufs[2] = {reinterpret_cast<float *>(base), reinterpret_cast<float *>(base) + buf_floats};

    const float *src = X0;
    int64_t lds = ldx;
    int next = 0;
    if (needs_pad(ldx, X0)) {  // 128-B aligned copy of X_0 (workspace buffer 0)
        const int rc = sgc_pad_rows_f32(X0, ldx, bufs[0], ldw, n_rows, F, stream);
        if (rc) return rc;
        src = bufs[0];
        lds = ldw;
        next = 1;
    }
    for (int h = 0; h < K; ++h) {
        const bool last = h == K - 1;
        float *dst = last ? out : bufs[next];
        const int64_t ldd = last ? ldo : ldw;
        // the workspace buffers' pad columns [F, ldw) may be read and written
        const uint32_t fl = (src != X0 ? SGC_SPMM_X_PADDED : 0u) | (last ? 0u : SGC_SPMM_Y_PADDED) |
                            (n_rows < (int64_t(1) << 24) && n_rows * lds * 4 < (int64_t(1) << 32)
                                 ? SGC_SPMM_X_UNDER_4G : 0u);
        // column groups: group 0 plain, groups 1.. continue its chains
        for (int g = 0; g < groups; ++g) {
            const int32_t *plan = plans_host ? plans_host[g] : nullptr;
            const uint32_t gf = fl | (g ? (uint32_t)SGC_SPMM_ACCUMULATE : 0u) |
                                (plan && plan_flags_host ? plan_flags_host[g] : 0u);
            const int rc = launch_spmm(row_ptrs + (int64_t)g * (n_rows + 1), col_idx, val, 0,
                                       n_rows, src, lds, dst, ldd, F, plan,
                                       plan ? n_heavy_host[g] : 0, plan ? n_hub_host[g] : 0,
                                       plan ? thresholds_host[g] : 0, gf, s);
            if (rc) return rc;
        }
        src = dst;
        lds = ldd;
        next ^= 1;
    }
    return SGC_OK;
}

int sgc_propagate_f32(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                      int64_t n_rows, const float *X0, int64_t ldx, float *out, int64_t ldo,
                      int64_t F, int32_t K, const int32_t *plan, int64_t n_heavy, int64_t n_hub,
                      int32_t heavy_threshold, void *workspace, int64_t workspace_bytes,
                      void *stream) {
    const int32_t *plans[1] = {plan};
    return sgc_propagate_groups_f32(1, row_ptr, col_idx, val, n_rows, X0, ldx, out, ldo, F, K,
                                    plan ? plans : nullptr, &n_heavy, &n_hub, &heavy_threshold,
                                    nullptr, workspace, workspace_bytes, stream);
}

int sgc_linear_f32(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                   int64_t ldy, int64_t M, int64_t K, int64_t C, void *stream) {
    return launch_linear_f32(X, ldx, W, b, Y, ldy, M, K, C, as_stream(stream));
}

const char *sgc_linear_kernel_name(int64_t M, int64_t K, int64_t ldx, int64_t C, const float *X) {
    return linear_kernel_name(M, K, ldx, C, X);
}

const char *sgc_linear_backward_kernel_name(int64_t M, int64_t K, int64_t ldx, int64_t C,
                                            const float *X) {
    return linear_backward_kernel_name(M, K, ldx, C, X);
}

int64_t sgc_linear_backward_workspace(int64_t M, int64_t K, int64_t C) {
    return linear_backward_workspace_bytes(M, K, C);
}

int sgc_linear_backward_f32(const float *X, int64_t ldx, const float *dY, int64_t ldd, int64_t M,
                            int64_t K, int64_t C, float *dW, float *db, void *workspace,
                            int64_t workspace_bytes, void *stream) {
    return linear_backward_f32(X, ldx, dY, ldd, M, K, C, dW, db, workspace, workspace_bytes,
                               as_stream(stream));
}

int64_t sgc_cross_entropy_workspace(int64_t M, int64_t C) { return cross_entropy_workspace(M, C); }

int sgc_cross_entropy_f32(const float *logits, int64_t ldl, const int64_t *labels, int64_t M,
                          int64_t C, int64_t ignore_index, float *loss, float *inv_count,
                          float *lse, void *workspace, int64_t workspace_bytes, void *stream) {
    return cross_entropy_fwd_f32(logits, ldl, labels, M, C, ignore_index, loss, inv_count, lse,
                                 workspace, workspace_bytes, as_stream(stream));
}

int sgc_cross_entropy_backward_f32(const float *logits, int64_t ldl, const int64_t *labels,
                                   const float *lse, const float *inv_count,
                                   const float *grad_loss, int64_t M, int64_t C,
                                   int64_t ignore_index, float *dlogits, int64_t ldd, void *stream) {
    return cross_entropy_bwd_f32(logits, ldl, labels, lse, inv_count, grad_loss, M, C,
                                 ignore_index, dlogits, ldd, as_stream(stream));
}

int64_t sgc_linear_xent_workspace(int64_t M, int64_t K, int64_t C) {
    return xent_workspace_bytes(M, K, C);
}

int sgc_linear_xent_f32(const float *X, int64_t ldx, const float *W, const float *b,
                        const int64_t *labels, int64_t M, int64_t K, int64_t C, float *loss,
                        float *dW, float *db, float *logits, int64_t ldl, void *workspace,
                        int64_t workspace_bytes, void *stream) {
    return linear_xent_f32(X, ldx, W, b, labels, M, K, C, loss, dW, db, logits, ldl, workspace,
                           workspace_bytes, as_stream(stream));
}

int sgc_warmup(uint32_t units, void *stream) {
    SGC_REQUIRE((units & ~7u) == 0, SGC_EINVAL, "warmup: unknown unit bits 0x%x", units);
    hipStream_t s = as_stream(stream);
    if (units & SGC_WARM_PROPAGATE) {
        SGC_HIP_CHECK(warm_side_streams());  // the SpMM's side-stream pool
        SGC_HIP_CHECK(warm_spmm(s));
        SGC_HIP_CHECK(warm_ingest(s));
        SGC_HIP_CHECK(warm_plan(s));
        SGC_HIP_CHECK(warm_sort(s));
        SGC_HIP_CHECK(warm_groups(s));
        SGC_HIP_CHECK(warm_exchange(s));
    }
    if (units & SGC_WARM_CLASSIFIER) {
        SGC_HIP_CHECK(warm_linear(s));
        SGC_HIP_CHECK(warm_xent(s));
        SGC_HIP_CHECK(warm_loss(s));
    }
    if (units & SGC_WARM_LOADERS) {
        SGC_HIP_CHECK(warm_normalize(s));
        SGC_HIP_CHECK(warm_subgraph(s));
    }
    SGC_HIP_CHECK(hipStreamSynchronize(s));
    return SGC_OK;
}

int sgc_timing_enable(int on) { return timing_enable(on); }

int sgc_timing_collect(float *light_ms_host, float *hub_ms_host, int64_t capacity,
                       int64_t *n_host) {
    return timing_collect(light_ms_host, hub_ms_host, capacity, n_host);
}

int sgc_timing_collect_ex(float *light_ms_host, float *hub_ms_host, float *span_ms_host,
                          int32_t *light_kernel_host, int64_t capacity, int64_t *n_host) {
    return timing_collect_ex(light_ms_host, hub_ms_host, span_ms_host, light_kernel_host,
                             capacity, n_host);
}

/* ---- host (CPU) twins ---------------------------------------------------- */

int sgc_coo_to_csr_cpu(const int64_t *rows, const int64_t *cols, const float *vals, int64_t nnz,
                       int64_t n_rows, int64_t n_cols, int32_t *row_ptr, int32_t *col_idx,
                       float *val_out, uint32_t *status_host) {
    return coo_to_csr_cpu(rows, cols, vals, nnz, n_rows, n_cols, row_ptr, col_idx, val_out,
                          status_host);
}

int sgc_spmm_csr_f32_cpu(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                         int64_t row_begin, int64_t row_end, const float *X, int64_t ldx,
                         float *Y, int64_t ldy, int64_t F, int32_t n_threads) {
    return spmm_cpu(row_ptr, col_idx, val, row_begin, row_end, X, ldx, Y, ldy, F, n_threads,
                    false);
}

int sgc_spmm_csr_f32_cpu_ex(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                            int64_t row_begin, int64_t row_end, const float *X, int64_t ldx,
                            float *Y, int64_t ldy, int64_t F, uint32_t flags, int32_t n_threads) {
    // the padding flags only license wider GPU loads; the CPU reads exactly F
    constexpr uint32_t known = SGC_SPMM_X_PADDED | SGC_SPMM_Y_PADDED | SGC_SPMM_ACCUMULATE;
    SGC_REQUIRE((flags & ~known) == 0, SGC_EINVAL, "spmm_cpu_ex: unsupported flags 0x%x", flags);
    return spmm_cpu(row_ptr, col_idx, val, row_begin, row_end, X, ldx, Y, ldy, F, n_threads,
                    (flags & SGC_SPMM_ACCUMULATE) != 0);
}

int64_t sgc_propagate_cpu_workspace(int64_t n_rows, int64_t F, int32_t K) {
    return propagate_cpu_workspace(n_rows, F, K);
}

int sgc_propagate_f32_cpu(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                          int64_t n_rows, const float *X0, int64_t ldx, float *out, int64_t ldo,
                          int64_t F, int32_t K, void *workspace, int64_t workspace_bytes,
                          int32_t n_threads) {
    return propagate_cpu(row_ptr, col_idx, val, n_rows, X0, ldx, out, ldo, F, K, workspace,
                         workspace_bytes, n_threads);
}

}  // extern "C"

int sgc_mgpu_init(int ndev, const int *devices) { return mgpu_init(ndev, devices); }

int sgc_mgpu_attach(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                    int64_t n_rows, int64_t nnz, void *stream, int64_t *handle) {
    return mgpu_attach(row_ptr, col_idx, val, n_rows, nnz, as_stream(stream), handle);
}

int sgc_mgpu_propagate(int64_t handle, const float *X0, int64_t ldx, float *out, int64_t ldo,
                       int64_t F, int32_t K, void *stream) {
    return mgpu_propagate(handle, X0, ldx, out, ldo, F, K, as_stream(stream));
}

int sgc_mgpu_detach(int64_t handle) { return mgpu_detach(handle); }

int sgc_mgpu_finalize(void) { return mgpu_finalize(); }

int64_t sgc_colsplit_workspace(int64_t n_rows, int32_t groups) {
    return colsplit_workspace(n_rows, groups);
}

int sgc_csr_colsplit(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                     int64_t n_rows, int64_t n_cols, int32_t groups, const int32_t *cuts_host,
                     int32_t *row_ptrs, int32_t *col_out, float *val_out, void *workspace,
                     int64_t workspace_bytes, void *stream) {
    return colsplit(row_ptr, col_idx, val, n_rows, n_cols, groups, cuts_host, row_ptrs, col_out,
                    val_out, workspace, workspace_bytes, as_stream(stream));
}

int64_t sgc_plan_sorted_workspace(int64_t n_rows) { return plan_sorted_workspace(n_rows); }

int sgc_plan_sorted(const int32_t *row_ptr, int64_t row_begin, int64_t row_end,
                    int32_t threshold, int32_t hub_threshold, int32_t *plan, void *workspace,
                    int64_t workspace_bytes, int64_t *counts_host, void *stream) {
    return plan_sorted(row_ptr, row_begin, row_end, threshold, hub_threshold, plan, workspace,
                       workspace_bytes, counts_host, as_stream(stream));
}
