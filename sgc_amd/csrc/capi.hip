// capi.hip -- extern "C" entry points of libsgc_amd.so (include/sgc_amd.h).
#include <cstdarg>
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
               int32_t *plan, int64_t capacity, int64_t *n_heavy_host, hipStream_t stream);
int launch_spmm(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                int64_t row_begin, int64_t row_end, const float *X, int64_t ldx, float *Y,
                int64_t ldy, int64_t F, const int32_t *heavy_rows, int64_t n_heavy,
                int32_t heavy_threshold, hipStream_t stream);
int launch_linear_f32(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                      int64_t ldy, int64_t M, int64_t K, int64_t C, hipStream_t stream);

}  // namespace sgc

using namespace sgc;

extern "C" {

int sgc_abi_version(void) { return SGC_ABI_VERSION; }

const char *sgc_last_error(void) { return g_err; }

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

int64_t sgc_plan_capacity(int64_t n_rows) { return 2 * (n_rows < 0 ? 0 : n_rows) + 1; }

int sgc_plan_build(const int32_t *row_ptr, int64_t row_begin, int64_t row_end,
                   int32_t heavy_threshold, int32_t *plan, int64_t plan_capacity,
                   int64_t *n_heavy_host, void *stream) {
    return build_plan(row_ptr, row_begin, row_end, heavy_threshold, plan, plan_capacity,
                      n_heavy_host, as_stream(stream));
}

int sgc_spmm_csr_f32(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                     int64_t row_begin, int64_t row_end, const float *X, int64_t ldx, float *Y,
                     int64_t ldy, int64_t F, const int32_t *plan, int64_t n_heavy,
                     int32_t heavy_threshold, void *stream) {
    return launch_spmm(row_ptr, col_idx, val, row_begin, row_end, X, ldx, Y, ldy, F, plan,
                       plan ? n_heavy : 0, heavy_threshold, as_stream(stream));
}

int sgc_propagate_f32(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                      int64_t n_rows, const float *X0, int64_t ldx, float *out, int64_t ldo,
                      float *work, int64_t F, int32_t K, const int32_t *plan, int64_t n_heavy,
                      int32_t heavy_threshold, void *stream) {
    hipStream_t s = as_stream(stream);
    SGC_REQUIRE(K >= 0, SGC_EINVAL, "propagate: negative degree %d", K);
    SGC_REQUIRE(X0 && out, SGC_EINVAL, "propagate: null pointer");
    SGC_REQUIRE(K <= 1 || work, SGC_EINVAL, "propagate: K=%d needs a work buffer", K);
    if (K == 0) {
        if (n_rows > 0 && F > 0)
            SGC_HIP_CHECK(hipMemcpy2DAsync(out, ldo * 4, X0, ldx * 4, F * 4, n_rows,
                                           hipMemcpyDeviceToDevice, s));
        return SGC_OK;
    }
    const float *src = X0;
    int64_t lds = ldx;
    for (int h = 0; h < K; ++h) {
        const bool to_out = ((K - 1 - h) & 1) == 0;
        float *dst = to_out ? out : work;
        const int64_t ldd = to_out ? ldo : F;
        const int rc = launch_spmm(row_ptr, col_idx, val, 0, n_rows, src, lds, dst, ldd, F, plan,
                                   plan ? n_heavy : 0, heavy_threshold, s);
        if (rc) return rc;
        src = dst;
        lds = ldd;
    }
    return SGC_OK;
}

int sgc_linear_f32(const float *X, int64_t ldx, const float *W, const float *b, float *Y,
                   int64_t ldy, int64_t M, int64_t K, int64_t C, void *stream) {
    return launch_linear_f32(X, ldx, W, b, Y, ldy, M, K, C, as_stream(stream));
}

}  // extern "C"
