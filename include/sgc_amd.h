/*
 * sgc_amd.h -- C ABI of libsgc_amd.so, the MI355X (gfx950) propagation engine
 * behind SGC's sgc_precompute() / SGC.forward().
 *
 * The reference (bellaj09/SGC) has no native code and no FFI: its hot path is
 * three lines of Python calling torch (utils.py:92-97 -> torch.spmm at
 * utils.py:95; models.py:17-18 -> nn.Linear).  Each entry point below names
 * the reference call it replaces.  Conventions:
 *
 *   - every pointer is a DEVICE pointer unless the parameter name ends in
 *     _host; buffers are owned by the caller (torch), never freed here;
 *   - `stream` is a hipStream_t passed as void* (torch:
 *     torch.cuda.current_stream().cuda_stream); all work is enqueued
 *     asynchronously on it; nothing here synchronises the device except the
 *     calls documented as "synchronous";
 *   - return 0 on success, a positive SGC_E* code on failure;
 *     sgc_last_error() returns a thread-local message for the last failure;
 *   - thread safety: every entry point may be called from several host
 *     threads at once (on different streams); the SpMM's internal side
 *     stream (hub rows) is serialised per device so one call's fork/join
 *     never interleaves with another's;
 *   - indices are int32 (n_rows, n_cols, nnz < 2^31), values fp32.
 */
#ifndef SGC_AMD_H
#define SGC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGC_ABI_VERSION 1

enum {
    SGC_OK = 0,
    SGC_EINVAL = 1,   /* bad argument (shape, stride, alignment, null)   */
    SGC_ERANGE = 2,   /* size or index outside the int32 CSR limits      */
    SGC_EHIP = 3,     /* a HIP runtime call failed                       */
    SGC_ENOMEM = 4,   /* workspace too small                             */
    SGC_EDEVICE = 5   /* no gfx950 device / kernel image not loadable    */
};

int sgc_abi_version(void);
const char *sgc_last_error(void);

/* Process-wide schedule knobs (results never depend on them).
 *   "slice_floats": feature-slice width of the SpMM grid in floats (default
 *                   128 = one 64V-float chunk per slice; 0 = one slice as wide
 *                   as the registers allow);
 *   "max_vec":      widest per-lane load, 1, 2 or 4 floats (default 4);
 *   "hub_chunk":    features per hub-kernel workgroup, 32 or 64 (default 0 =
 *                   32 when F <= 192 and X rows are 128-B aligned, else 64);
 *   "hub_stream":   1 = hub kernel on a side stream, concurrent with the
 *                   light kernel; 2 = on the caller's stream before the light
 *                   kernel (serial, no cross-stream events); 0 = default: the
 *                   side stream unless the launch sets SGC_SPMM_HUB_SERIAL;
 *   "rows_per_wave": light rows per wavefront when 16-B lanes are possible
 *                   (0 = default, auto; 2 = 32 lanes x 4 floats per row; 4 =
 *                   16 lanes; 1 = one row per wave with the slice_floats /
 *                   max_vec scheme);
 *   "hub_loaders":  loader waves per hub workgroup, 15 (default) or 7;
 *   "hub_fuse":     1 (default) = serial hub rows (SGC_SPMM_HUB_SERIAL) run as
 *                   the first workgroups of the light kernel's own launch
 *                   (three loader waves + the chain wave each) where that is
 *                   the multi-row kernel over 16-B-lane slices or the
 *                   one-chunk csr kernel; 0 = their own launch before it;
 *   "heavy_pairs":  heavy-row load forms, a bit mask (default 29): 1 pairs in
 *                   the multi-row kernel, 2 in the one-row kernel, 4 four
 *                   nonzeros per load up to 32 floats, 8 the same transposed
 *                   at 33..64 floats, 16 the pairs transposed;
 *   "tile_buffers": classifier LDS tile images, 1 (default) or 2;
 *   "linear_kernel": classifier forward, 0 = auto (the streaming kernel where
 *                   W^T fits LDS and M >= 4096), 1 = LDS tile, 2 = streaming
 *                   (3 / 4: its diagnostic forms -- loads only / MFMAs only --
 *                   whose results are wrong by design);
 *   "linear_ck":    k per chunk of the streaming forward, 64 (default) or 32;
 *   "backward_kernel": classifier weight backward, 0 = auto (split-bf16
 *                   column blocks up to 48 classes, else the fp32 MFMA
 *                   slabs), 1 = fp32 MFMA slabs, 2 = split-bf16 slabs where X
 *                   gives 8-B lanes (K and ldx even), 3 = split-bf16 column
 *                   blocks (up to 48 classes; more: as 0).
 * sgc_get_tuning returns -1 for an unknown key. */
int sgc_set_tuning(const char *key, int64_t value);
int64_t sgc_get_tuning(const char *key);

/* ---------------------------------------------------------------------------
 * Ingest: torch sparse COO -> CSR.
 * Replaces the implicit COO handling inside torch.spmm (utils.py:95) for the
 * adjacency built by sparse_mx_to_torch_sparse_tensor (utils.py:23-30:
 * int64 [2,nnz] indices, fp32 values).  The CSR keeps every stored entry
 * (no coalescing) and, within a row, the COO storage order (stable by row),
 * which is the order torch's CPU kernel applies its FMAs in.
 *
 * sgc_coo_to_csr_workspace: bytes of device scratch sgc_coo_to_csr needs.
 * sgc_coo_to_csr: rows/cols are the two rows of the [2,nnz] index tensor.
 *   status_host (synchronous; may be NULL to stay asynchronous) receives a
 *   bit set: 1 = input rows already sorted, 2 = every CSR row has strictly
 *   ascending columns, 4 = an index was out of range (CSR then invalid).
 * ------------------------------------------------------------------------- */
int sgc_coo_to_csr_workspace(int64_t n_rows, int64_t nnz, size_t *bytes_host);
int sgc_coo_to_csr(const int64_t *rows, const int64_t *cols, const float *vals,
                   int64_t nnz, int64_t n_rows, int64_t n_cols,
                   int32_t *row_ptr, int32_t *col_idx, float *val_out,
                   void *workspace, size_t workspace_bytes,
                   uint32_t *status_host, void *stream);

/* Same, from torch CSR (crow_indices/col_indices int64): narrows to int32. */
int sgc_csr64_to_csr(const int64_t *crow, const int64_t *col, const float *vals,
                     int64_t nnz, int64_t n_rows, int64_t n_cols,
                     int32_t *row_ptr, int32_t *col_idx, float *val_out,
                     uint32_t *status_host, void *stream);

/* ---------------------------------------------------------------------------
 * On-device augmented normalisation S = D^-1/2 (A+I) D^-1/2 (reference
 * normalization.py:5-12 + the fp32 rounding of utils.py:25), bit-exact with
 * scipy's result.  A: canonical CSR (ascending unique columns per row), fp64
 * values.  Two passes around one host step, exactly as the reference splits
 * its arithmetic:
 *   1. sgc_augnorm_count: per-row entry count of A+I -> out_row_ptr (scan) and
 *      rowsum (fp64, sequential in column order); *out_nnz_host = nnz(S).
 *      Synchronous.  Returns SGC_EINVAL if A is not canonical.
 *   2. host: d = rowsum ** -0.5, inf -> 0 (numpy, as normalization.py:8-10);
 *   3. sgc_augnorm_fill: S entries (d_i * a_ij) * d_j in fp64 -> fp32, in
 *      ascending column order, dropping exact zeros like scipy's csr_matmat
 *      (out_row_ptr may shrink then; *out_nnz_host = final nnz).  Synchronous.
 * workspace: sgc_augnorm_workspace(n) bytes of device scratch.
 * ------------------------------------------------------------------------- */
int64_t sgc_augnorm_workspace(int64_t n_rows);
int sgc_augnorm_count(const int32_t *row_ptr, const int32_t *col_idx, const double *val,
                      int64_t n_rows, int64_t nnz, int32_t *out_row_ptr, double *rowsum,
                      void *workspace, int64_t workspace_bytes, int64_t *out_nnz_host,
                      uint32_t *status_host, void *stream);
int sgc_augnorm_fill(const int32_t *row_ptr, const int32_t *col_idx, const double *val,
                     int64_t n_rows, const double *d, int32_t *out_row_ptr,
                     int32_t *out_col_idx, float *out_val, void *workspace,
                     int64_t workspace_bytes, int64_t *out_nnz_host, void *stream);

/* ---------------------------------------------------------------------------
 * Induced sub-graph B = A[idx][:, idx] (reference utils.py:117, the inductive
 * train sub-graph of reddit.py:44-47, taken on A + A^T before normalisation).
 * A: CSR (int32), fp64 values; idx: int64 [m], distinct ids in [0, n_rows).
 * B: canonical CSR (new row i = old row idx[i], new column = position in
 * idx, ascending), fp64 values -- the input sgc_augnorm_count/fill take, so
 * the S_train built from B is the reference's bit for bit.  Two synchronous
 * calls around the host allocation of B, sharing one workspace:
 *   sgc_subgraph_count: out_row_ptr [m+1], *out_nnz_host = nnz(B);
 *     status_host bits: 1 = repeated ids (SGC_EINVAL), 2 = idx ascending,
 *     4 = an id out of range (SGC_ERANGE);
 *   sgc_subgraph_fill: out_col_idx / out_val [nnz(B)].
 * workspace: sgc_subgraph_workspace(n_rows, m, nnz(A)) bytes.
 * ------------------------------------------------------------------------- */
int64_t sgc_subgraph_workspace(int64_t n_rows, int64_t m, int64_t nnz);
int sgc_subgraph_count(const int32_t *row_ptr, const int32_t *col_idx, int64_t n_rows,
                       int64_t nnz, const int64_t *idx, int64_t m, int32_t *out_row_ptr,
                       void *workspace, int64_t workspace_bytes, int64_t *out_nnz_host,
                       uint32_t *status_host, void *stream);
int sgc_subgraph_fill(const int32_t *row_ptr, const int32_t *col_idx, const double *val,
                      int64_t n_rows, int64_t nnz, const int64_t *idx, int64_t m,
                      const int32_t *out_row_ptr, int32_t *out_col_idx, double *out_val,
                      void *workspace, int64_t workspace_bytes, void *stream);

/* CSR -> torch COO indices: rows64[k], cols64[k] (int64) of every entry. */
int sgc_csr_to_coo64(const int32_t *row_ptr, const int32_t *col_idx, int64_t n_rows,
                     int64_t *rows64, int64_t *cols64, void *stream);

/* ---------------------------------------------------------------------------
 * Schedule ("plan") for the SpMM.  Lists the rows of [row_begin, row_end)
 * with more than heavy_threshold nonzeros, heaviest first; the first n_hub
 * of them have more than hub_threshold (>= heavy_threshold).
 * sgc_spmm_csr_f32 runs
 *   - each hub row on 1024-thread workgroups (one per 64-feature chunk; 15
 *     waves gather nonzeros ahead into LDS, one runs the FMA chain), on a
 *     side stream joined back to the caller's stream;
 *   - each other heavy row as one wave per 128-float chunk, scheduled first;
 *   - every remaining row as one wave.
 * The plan changes only the schedule: every output element is still one
 * sequential FMA chain, so results never depend on it.  Synchronous (reads
 * the heavy-row list back to sort it).
 *
 * plan must hold sgc_plan_capacity(row_end - row_begin) int32 words;
 * *n_heavy_host receives the number of heavy rows written to plan[0..),
 * *n_hub_host (may be NULL) how many of them lead as hub rows.
 * ------------------------------------------------------------------------- */
int64_t sgc_plan_capacity(int64_t n_rows);
int sgc_plan_build(const int32_t *row_ptr, int64_t row_begin, int64_t row_end,
                   int32_t heavy_threshold, int32_t hub_threshold, int32_t *plan,
                   int64_t plan_capacity, int64_t *n_heavy_host, int64_t *n_hub_host,
                   void *stream);
/* The light rows' processing order for SGC_SPMM_LIGHT_ORDER: every row of
 * [row_begin, row_end) with at most heavy_threshold nonzeros, longest first,
 * ties in row order (a stable counting sort on the host after one read-back
 * of row_ptr), written to light[0 .. *n_light_host) on the device (light
 * must hold row_end - row_begin words); synchronous on `stream`.  Place it
 * after the n_heavy rows of sgc_plan_build's plan.  A schedule only. */
int sgc_plan_light_order(const int32_t *row_ptr, int64_t row_begin, int64_t row_end,
                         int32_t heavy_threshold, int32_t *light, int64_t *n_light_host,
                         void *stream);

/* ---------------------------------------------------------------------------
 * One hop Y = S[row_begin:row_end, :] . X  (utils.py:95, torch.spmm).
 * Y row 0 receives S row row_begin.  Each Y[i,f] is
 *     acc = +0.0f; for k in row i (CSR order): acc = fmaf(val[k], X[col[k], f], acc)
 * -- bit-identical to the reference CPU kernel.  X rows have stride ldx
 * floats, Y rows ldy floats; X must not alias Y.
 * plan/n_heavy/n_hub/heavy_threshold from sgc_plan_build over the same row
 * range, or plan = NULL (one work item per row, natural order).
 * ------------------------------------------------------------------------- */
int sgc_spmm_csr_f32(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                     int64_t row_begin, int64_t row_end,
                     const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                     const int32_t *plan, int64_t n_heavy, int64_t n_hub,
                     int32_t heavy_threshold, void *stream);

/* Per-kernel launch timing (diagnostics; off by default).  While enabled,
 * every sgc_spmm_csr_f32 records timing events around its light/heavy-row
 * kernel and around its hub-row kernel, each on the stream that kernel runs
 * on.  sgc_timing_collect waits for the recorded launches (synchronous) and
 * writes, in launch order, light_ms_host[i] and hub_ms_host[i] (-1 when the
 * launch had no hub rows); *n_host = launches recorded since the last
 * collect (SGC_ENOMEM when capacity is smaller; nothing is consumed then).
 * Do not enable while capturing a graph. */
int sgc_timing_enable(int on);
int sgc_timing_collect(float *light_ms_host, float *hub_ms_host, int64_t capacity,
                       int64_t *n_host);
/* Same, plus per launch: span_ms_host[i] = the whole launch (first kernel
 * start to the later kernel end: what the caller's stream waits for) and
 * light_kernel_host[i] = which light/heavy-row kernel ran (0 spmm_csr_kernel,
 * 1 spmm_rows_kernel, 2 / 3 spmm_rows_kernel / spmm_csr_kernel with the
 * serial hub rows fused into its launch, -1 none: a hub-only launch).  Either
 * may be NULL. */
int sgc_timing_collect_ex(float *light_ms_host, float *hub_ms_host, float *span_ms_host,
                          int32_t *light_kernel_host, int64_t capacity, int64_t *n_host);

/* Same, with flags.
 * Layout, for buffers whose rows are padded (the engine's own 128-B-row
 * buffers): SGC_SPMM_X_PADDED = X's columns [F, round4(F)) are allocated in
 * every row and may be read (their values do not matter); SGC_SPMM_Y_PADDED
 * = Y's columns [F, round4(F)) are allocated and may be overwritten with
 * don't-care values.  They let the kernel use 16-B lanes at any F; columns
 * < F are bit-identical either way.
 * Split launch of one hop (the multi-GPU pipeline runs the hub rows beside
 * several narrower launches): SGC_SPMM_NO_HUB = skip the plan's n_hub hub
 * rows (their Y rows are not written); SGC_SPMM_HUB_ONLY = only the hub rows,
 * on `stream` itself (no side stream).  The two launches together write
 * exactly what one unflagged launch writes.
 * Column-block passes (the multi-GPU pipeline that consumes an exchange in
 * column order, sgc_amd.distributed.CyclicRowPropagator): SGC_SPMM_ACCUMULATE
 * = each element's FMA chain starts from Y's current value instead of +0.0f,
 * and rows without nonzeros in this CSR are left untouched.  When S's
 * nonzeros are split by column range into CSRs S_0, S_1, ... (each row's
 * nonzeros of S_g precede those of S_{g+1} in CSR order), one unflagged
 * launch over S_0 followed by ACCUMULATE launches over S_1, S_2, ... writes
 * exactly what one launch over S writes (the fp32 store/load between passes
 * is exact).
 * SGC_SPMM_HUB_SERIAL: run the hub rows' kernel on `stream` before the light
 * kernel instead of beside it on a side stream (no fork/join events); for
 * launches whose longest hub chain is shorter than the ~20-30 us a
 * cross-stream fork/join costs (sgc_set_tuning "hub_stream" overrides).
 * SGC_SPMM_LIGHT_ORDER: `plan` holds row_end - row_begin entries: its n_heavy
 * heavy rows (as sgc_plan_build writes them) followed by every other row of
 * the range, in the order the light rows are to be processed (the Python
 * layer sorts them by length, so the rows sharing a wavefront in the
 * multi-row kernel have about the same length and few lanes idle-load past
 * their row's end).  A schedule only: results never depend on it.
 * SGC_SPMM_X_UNDER_4G: the caller vouches that X has fewer than 2^24 rows
 * and that every X row a column id can name lies within 4 GiB of X
 * (n_cols * ldx * 4 < 2^32), so the gathers may use 32-bit row offsets from
 * one 24-bit multiply (fewer address instructions per nonzero).  The library
 * cannot check it (it never sees n_cols here): a caller that sets the flag
 * for a larger X gets wrapped addresses -- wrong rows gathered -- not an
 * error.  sgc_propagate_f32 / sgc_propagate_groups_f32 and the Python layer
 * derive it themselves from n_rows and the row stride.  */
enum { SGC_SPMM_X_PADDED = 1, SGC_SPMM_Y_PADDED = 2, SGC_SPMM_NO_HUB = 4,
       SGC_SPMM_HUB_ONLY = 8, SGC_SPMM_ACCUMULATE = 16, SGC_SPMM_HUB_SERIAL = 32,
       SGC_SPMM_LIGHT_ORDER = 64, SGC_SPMM_X_UNDER_4G = 128 };
int sgc_spmm_csr_f32_ex(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                        int64_t row_begin, int64_t row_end,
                        const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                        const int32_t *plan, int64_t n_heavy, int64_t n_hub,
                        int32_t heavy_threshold, uint32_t flags, void *stream);

/* K hops X_K = S^K X_0 over all n_rows rows (utils.py:92-97, the whole
 * sgc_precompute loop).  out (row stride ldo) receives X_K.  Intermediate
 * hops live in the workspace with 128-B aligned rows (ld = F rounded up to 32
 * floats: a gathered X row segment then spans the fewest 128-B lines); when
 * X_0's rows are not 128-B aligned it is first copied into that layout
 * (sgc_pad_rows_f32), which costs one streaming copy and saves ~9% per hop
 * that reads it at Reddit shape.  K = 0 copies X_0 into out (the Python
 * layer returns the input object itself, as the reference does).
 * sgc_propagate_workspace: bytes of device workspace for these arguments. */
int64_t sgc_propagate_workspace(int64_t n_rows, int64_t F, int64_t ldx, int32_t K);
int sgc_propagate_f32(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                      int64_t n_rows, const float *X0, int64_t ldx, float *out,
                      int64_t ldo, int64_t F, int32_t K,
                      const int32_t *plan, int64_t n_heavy, int64_t n_hub,
                      int32_t heavy_threshold, void *workspace, int64_t workspace_bytes,
                      void *stream);

/* The same loop over S split into `groups` column groups (sgc_csr_colsplit:
 * row_ptrs [groups][n_rows+1] absolute into one col_idx / val pair; rows with
 * ascending columns), each hop as `groups` launches -- group 0 plain, groups
 * 1.. with SGC_SPMM_ACCUMULATE -- which is bit-identical to one launch per
 * hop and faster at Reddit shape.  Per group g:
 * plans_host[g] / n_heavy_host[g] / n_hub_host[g] / thresholds_host[g] =
 * sgc_plan_sorted over group g's CSR (plans_host NULL = no plans), and
 * plan_flags_host[g] (may be NULL) = SGC_SPMM_LIGHT_ORDER (plans_host[g]
 * lists every row, as sgc_plan_sorted writes it) | SGC_SPMM_HUB_SERIAL.
 * groups = 1 with row_ptrs = the CSR's row_ptr is sgc_propagate_f32 with
 * plan flags.  Same workspace as sgc_propagate_f32. */
int sgc_propagate_groups_f32(int32_t groups, const int32_t *row_ptrs, const int32_t *col_idx,
                             const float *val, int64_t n_rows, const float *X0, int64_t ldx,
                             float *out, int64_t ldo, int64_t F, int32_t K,
                             const int32_t *const *plans_host, const int64_t *n_heavy_host,
                             const int64_t *n_hub_host, const int32_t *thresholds_host,
                             const uint32_t *plan_flags_host, void *workspace,
                             int64_t workspace_bytes, void *stream);

/* Row-strided copy dst[i, 0:F] = src[i, 0:F] (re-layout of feature rows). */
int sgc_pad_rows_f32(const float *src, int64_t lds, float *dst, int64_t ldd,
                     int64_t n_rows, int64_t F, void *stream);

/* Batched 2-D block copy, one launch (the multi-GPU exchanges' unpack,
 * sgc_amd.distributed): for each of nseg <= 64 segments, segs_host[6s ..
 * 6s+5] = (src_row, src_col, dst_row, dst_col, rows, cols):
 *     dst[dst_row + i, dst_col + j] = src[src_row + i, src_col + j],
 * i < rows, j < cols; row strides lds / ldd (floats).  Segments must not
 * overlap in dst.  Replaces the P strided copies that landed each rank's
 * column block of an all-gathered row chunk in X_K (the reference returns the
 * whole X_K from utils.py:92-97, so every rank needs all of it). */
int sgc_copy_blocks_f32(const float *src, int64_t lds, float *dst, int64_t ldd, int32_t nseg,
                        const int64_t *segs_host, void *stream);

/* Peer exchange over IPC-mapped memory: the replicated output of the
 * partitioned sgc_precompute (utils.py:92-97 returns all of X_K to every
 * caller) without a gathered copy.  Each rank exposes one buffer of its own
 * (its last hop's column blocks + int32 flags); the peers map it once and
 * every call (1) computes a row chunk into that buffer, (2) raises the chunk's
 * flag to the call's sequence number (sgc_signal_flag_i32), (3) waits for every
 * peer's flag (sgc_wait_flags_i32) and (4) pulls all P blocks of the chunk
 * straight into X_K's columns (sgc_pull_blocks_f32).
 *
 * sgc_ipc_get_handle: the SGC_IPC_HANDLE_BYTES handle of the allocation that
 * holds `ptr` (hipIpcGetMemHandle) with ptr's offset in it.  sgc_ipc_open (in
 * another process): maps it; *base_host is what sgc_ipc_close takes, *ptr_host
 * the peer's pointer in this process. */
#define SGC_IPC_HANDLE_BYTES 128
int sgc_ipc_get_handle(const void *ptr, void *handle_host);
int sgc_ipc_open(const void *handle_host, void **base_host, void **ptr_host);
int sgc_ipc_close(void *base);
/* *flag = value once everything enqueued on `stream` before it is visible at
 * system scope (one-lane release store). */
int sgc_signal_flag_i32(int32_t *flag, int32_t value, void *stream);
/* The stream waits until flag_ptrs_host[i][0] >= value for every i < n (n <=
 * 64; one polling wave, acquire loads at system scope); after timeout_us it
 * stops waiting and sets *err = 1 (a host-visible word the caller checks after
 * synchronising: a lost peer never hangs the device). */
int sgc_wait_flags_i32(int32_t n, const int64_t *flag_ptrs_host, int32_t value, int32_t *err,
                       int64_t timeout_us, void *stream);
/* Batched 2-D block copy with one source pointer per segment (a peer's mapped
 * buffer or this rank's own): segs_host[6s .. 6s+5] = (src pointer, src row
 * stride in floats, dst_row, dst_col, rows, cols), nseg <= 16:
 *     dst[dst_row + i, dst_col + j] = src[i * lds + j];
 * sources read with system-coherent loads; a segment's source span must stay
 * below 2 GiB (split its rows). */
int sgc_pull_blocks_f32(int32_t nseg, const int64_t *segs_host, float *dst, int64_t ldd,
                        void *stream);

/* Recorded launch lists: the K-hop loop's launches (sgc_spmm_csr_f32_ex /
 * sgc_pad_rows_f32 with their arguments) recorded once and replayed by ONE
 * call per propagation -- at Pubmed shape the per-launch host cost (~4 us)
 * is a tenth of a hop.  A pointer argument of a recorded launch is either
 * fixed (SGC_SLOT_FIXED: the recorded pointer, e.g. an intermediate buffer the
 * caller keeps alive) or the run's X_0 / X_K (SGC_SLOT_X0 / SGC_SLOT_OUT: the
 * pointers given to sgc_launch_list_run), so one list serves every feature
 * tensor of the recorded shape, strides and alignment; each replayed launch
 * makes its kernel choice from the actual pointers, as a direct call does.
 * A list belongs to the device current at creation (the run switches to it
 * and back).  Runs, adds and destroys are serialised by one library lock
 * (a run is a few launches); one list must still not run concurrently on
 * two streams when it holds fixed intermediates.  No reference counterpart: the reference's
 * loop (utils.py:94-96) is one torch.spmm call per hop. */
enum { SGC_SLOT_FIXED = 0, SGC_SLOT_X0 = 1, SGC_SLOT_OUT = 2 };
int sgc_launch_list_create(int64_t *handle_host);
int sgc_launch_list_add_spmm(int64_t handle, const int32_t *row_ptr, const int32_t *col_idx,
                             const float *val, int64_t row_begin, int64_t row_end,
                             const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                             const int32_t *plan, int64_t n_heavy, int64_t n_hub,
                             int32_t heavy_threshold, uint32_t flags, int32_t x_slot,
                             int32_t y_slot);
int sgc_launch_list_add_pad_rows(int64_t handle, const float *src, int64_t lds, float *dst,
                                 int64_t ldd, int64_t n_rows, int64_t F, int32_t src_slot,
                                 int32_t dst_slot);
int sgc_launch_list_run(int64_t handle, const float *X0, float *out, void *stream);
int sgc_launch_list_destroy(int64_t handle);

/* The row stride (floats) the engine uses for its own feature buffers. */
int64_t sgc_aligned_ld(int64_t F);

/* ---------------------------------------------------------------------------
 * Classifier forward Y[M,C] = X[M,K] . W[C,K]^T + b[C]  (models.py:17-18,
 * nn.Linear) at fp32 precision on MFMA: where W's three bf16 images fit LDS
 * (e.g. K = 602, C <= 42) and M >= 4096, every operand is split exactly into
 * three bf16 pieces and the six products that reach fp32 precision run on
 * v_mfma_f32_16x16x32_bf16; otherwise fp32 MFMA (v_mfma_f32_16x16x4_f32).
 * b may be NULL.  X row stride ldx, Y row stride ldy.  Tolerance-equal to
 * torch (summation order differs), not bit-equal.
 * ------------------------------------------------------------------------- */
int sgc_linear_f32(const float *X, int64_t ldx, const float *W, const float *b,
                   float *Y, int64_t ldy, int64_t M, int64_t K, int64_t C, void *stream);

/* Name of the kernel sgc_linear_f32 launches for these arguments (under the
 * current "linear_kernel" tuning), for benchmark labels; "none" for an empty
 * or invalid shape.  Static storage. */
const char *sgc_linear_kernel_name(int64_t M, int64_t K, int64_t ldx, int64_t C, const float *X);
/* The weight-backward kernel sgc_linear_backward_f32 runs for this shape /
 * alignment under the current "backward_kernel" tuning (static string; bench
 * labels); "none" for an empty or invalid shape. */
const char *sgc_linear_backward_kernel_name(int64_t M, int64_t K, int64_t ldx, int64_t C,
                                            const float *X);

/* Backward of sgc_linear_f32 for the weights (what autograd runs for
 * nn.Linear after F.cross_entropy(model(x), y).backward() in the closures of
 * citation.py:47-49 and reddit.py:55-58):  dW[C,K] = dY^T X,  db[C] = sum_m dY
 * (db may be NULL), from one read of X on fp32 MFMA; dY [M,C] with row stride
 * ldd.  C <= 64.  Fixed-order reductions: bitwise reproducible run to run,
 * within fp32 tolerance of torch.  workspace: sgc_linear_backward_workspace
 * (M, K, C) bytes.  (dX = dY W, needed only when x requires a gradient, is
 * not computed here.) */
int64_t sgc_linear_backward_workspace(int64_t M, int64_t K, int64_t C);
int sgc_linear_backward_f32(const float *X, int64_t ldx, const float *dY, int64_t ldd,
                            int64_t M, int64_t K, int64_t C, float *dW, float *db,
                            void *workspace, int64_t workspace_bytes, void *stream);

/* Softmax cross-entropy over a logits matrix: the loss the reference's
 * closures take of the classifier's output, F.cross_entropy(model(x), y)
 * with mean reduction (citation.py:46-49, reddit.py:55-58), and its
 * gradient.  logits [M, C] (row stride ldl, C <= 64), labels int64 [M]; rows
 * whose label equals ignore_index are left out of the mean (torch's
 * default is -100).  Forward: *loss = mean over the counted rows of
 * lse_m - logits[m, y_m], lse[m] = log sum_c exp(logits[m, c]) (kept for the
 * backward), *inv_count = 1 / (counted rows); NaN loss for a label outside
 * [0, C).  Backward: dlogits = (softmax - onehot) * (*grad_loss) *
 * (*inv_count) (grad_loss may be NULL: 1), zero rows for ignored labels.
 * Device scalars throughout (no host synchronisation).  Deterministic;
 * tolerance-equal to torch (rtol 1e-5).  workspace:
 * sgc_cross_entropy_workspace(M, C) bytes. */
int64_t sgc_cross_entropy_workspace(int64_t M, int64_t C);
int sgc_cross_entropy_f32(const float *logits, int64_t ldl, const int64_t *labels, int64_t M,
                          int64_t C, int64_t ignore_index, float *loss, float *inv_count,
                          float *lse, void *workspace, int64_t workspace_bytes, void *stream);
int sgc_cross_entropy_backward_f32(const float *logits, int64_t ldl, const int64_t *labels,
                                   const float *lse, const float *inv_count,
                                   const float *grad_loss, int64_t M, int64_t C,
                                   int64_t ignore_index, float *dlogits, int64_t ldd, void *stream);

/* ---------------------------------------------------------------------------
 * Fused classifier training step: for the SGC closure
 * (citation.py:46-49, reddit.py:55-58: F.cross_entropy(model(x), y) then
 * backward) computes, in three launches reading X twice,
 *     loss = mean_m [ logsumexp(z_m) - z_m[y_m] ],  z = X W^T + b
 *     dW   = (softmax(z) - onehot(y))^T X / M,     db = sum_m (...) / M
 * loss is one float; dW [C,K], db [C] (db may be NULL); logits [M,C] with row
 * stride ldl are written when non-NULL.  C <= 64.  Labels must lie in
 * [0, C) (not checked on the device; the Python layer checks them).  Reductions run in a fixed order:
 * results are bitwise reproducible run to run; within fp32 tolerance of torch.
 * workspace: sgc_linear_xent_workspace(M, K, C) bytes.
 * ------------------------------------------------------------------------- */
int64_t sgc_linear_xent_workspace(int64_t M, int64_t K, int64_t C);
int sgc_linear_xent_f32(const float *X, int64_t ldx, const float *W, const float *b,
                        const int64_t *labels, int64_t M, int64_t K, int64_t C, float *loss,
                        float *dW, float *db, float *logits, int64_t ldl, void *workspace,
                        int64_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Host (CPU) twins, for CPU tensors: the reference runs utils.py:92-97 on the
 * CPU whenever CUDA is off (args.py:39 --no-cuda; load_citation(cuda=False)).
 * Every pointer here is a HOST pointer; the calls are synchronous and
 * thread-safe (no shared state).  Same numerical contract as the GPU entry
 * points: bit-identical to torch.spmm's CPU kernel.  n_threads <= 0 = all
 * hardware threads; threads own whole rows.
 *
 * sgc_coo_to_csr_cpu: as sgc_coo_to_csr (stable by row, no coalescing;
 *   status bits 1/2/4), SGC_ERANGE on an out-of-range index.
 * sgc_spmm_csr_f32_cpu: as sgc_spmm_csr_f32 (utils.py:95), no plan.
 * sgc_spmm_csr_f32_cpu_ex: with flags; SGC_SPMM_ACCUMULATE as on the GPU,
 *   the padding flags accepted (and unused), the hub-split flags rejected.
 * sgc_propagate_f32_cpu: as sgc_propagate_f32 (utils.py:92-97); workspace
 *   = sgc_propagate_cpu_workspace(n_rows, F, K) bytes of host memory.
 * ------------------------------------------------------------------------- */
int sgc_coo_to_csr_cpu(const int64_t *rows, const int64_t *cols, const float *vals,
                       int64_t nnz, int64_t n_rows, int64_t n_cols,
                       int32_t *row_ptr, int32_t *col_idx, float *val_out,
                       uint32_t *status_host);
int sgc_spmm_csr_f32_cpu(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                         int64_t row_begin, int64_t row_end,
                         const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                         int32_t n_threads);
int sgc_spmm_csr_f32_cpu_ex(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                            int64_t row_begin, int64_t row_end,
                            const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                            uint32_t flags, int32_t n_threads);
int64_t sgc_propagate_cpu_workspace(int64_t n_rows, int64_t F, int32_t K);
int sgc_propagate_f32_cpu(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                          int64_t n_rows, const float *X0, int64_t ldx, float *out,
                          int64_t ldo, int64_t F, int32_t K, void *workspace,
                          int64_t workspace_bytes, int32_t n_threads);

/* The whole launch plan in one call, on the device: plan[0 .. n) = every row
 * of [row_begin, row_end) sorted by degree, longest first, ties in ascending
 * row order (a stable radix sort) -- i.e. the heavy rows (degree > threshold)
 * heaviest first followed by the light rows in SGC_SPMM_LIGHT_ORDER order,
 * exactly what sgc_plan_build + sgc_plan_light_order write together.
 * counts_host[0] = rows above threshold (n_heavy), [1] = rows above
 * hub_threshold (n_hub), [2] = the longest row's nonzeros.  Synchronous (two
 * stream synchronisations: the counts, then the sort); workspace of
 * sgc_plan_sorted_workspace(n) bytes on the device.  Replaces nothing in the
 * reference (a schedule). */
int64_t sgc_plan_sorted_workspace(int64_t n_rows);
int sgc_plan_sorted(const int32_t *row_ptr, int64_t row_begin, int64_t row_end,
                    int32_t threshold, int32_t hub_threshold, int32_t *plan, void *workspace,
                    int64_t workspace_bytes, int64_t *counts_host, void *stream);

/* ---------------------------------------------------------------------------
 * Column groups of S (a schedule for the SpMM of utils.py:95; results
 * unchanged).  Splits every row's nonzeros at the column cuts
 * 0 = cuts[0] <= cuts[1] <= ... <= cuts[G] = n_cols into G CSRs over the same
 * rows.  REQUIRES rows whose columns do not decrease (sgc_coo_to_csr status
 * bit 2): group g's part of a row is then one contiguous run, the runs come
 * in group order, and a hop computed as G launches -- group 0 plain, groups
 * 1.. with SGC_SPMM_ACCUMULATE -- applies every row's FMAs in CSR order: the
 * same bits as one launch, while each launch gathers only its group's X rows
 * (a live X slice 1/G as large, more of it in the per-XCD L2s).
 *   row_ptrs: [G][n_rows+1] int32, group g's row_ptr at row_ptrs + g*(n_rows+1),
 *             absolute offsets into col_out/val_out (groups stored one after
 *             the other), so (row_ptrs + g*(n_rows+1), col_out, val_out) is an
 *             ordinary CSR for sgc_spmm_csr_f32_ex / sgc_plan_sorted;
 *   col_out / val_out: [nnz];  G <= 8;  asynchronous on `stream`;
 *   workspace: sgc_colsplit_workspace(n_rows, G) bytes on the device.
 * ------------------------------------------------------------------------- */
int64_t sgc_colsplit_workspace(int64_t n_rows, int32_t groups);
int sgc_csr_colsplit(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                     int64_t n_rows, int64_t n_cols, int32_t groups, const int32_t *cuts_host,
                     int32_t *row_ptrs, int32_t *col_out, float *val_out, void *workspace,
                     int64_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * One process, several GPUs (the multi-GPU form of the one
 * call reddit.py:43 makes, sgc_precompute -> utils.py:92-97).  The engine
 * splits the feature columns over the devices: device d pulls its column
 * block of X_0 from the home device (peer reads over xGMI), runs all K hops
 * over its own replica of S (no exchange between hops: column f of X_{k+1}
 * depends on column f of X_k only) and stores its block of X_K straight into
 * `out` on the home device.  Bit-identical to sgc_propagate_f32.
 *   sgc_mgpu_init(ndev, devices): devices[0] = home device (where the CSR,
 *     X_0 and out live); enables peer access between every pair, one stream
 *     per entry.  An index may repeat (virtual devices sharing one GPU).
 *     Re-initialising frees the previous engine and its attachments.
 *   sgc_mgpu_attach: replicate the CSR (home-device pointers, n_rows square)
 *     to every other device -- synchronous, once per adjacency -- and return
 *     a handle.  The caller keeps the home arrays alive until detach.
 *   sgc_mgpu_propagate: X_K = S^K X_0 (K >= 1) into out (row stride ldo),
 *     asynchronous on `stream` (home device): every device waits for the work
 *     already on `stream`, and `stream` waits for every device.
 *   sgc_mgpu_detach / sgc_mgpu_finalize: free one attachment / everything.
 * Replaces: the torch.spmm loop of utils.py:94-95 spread over the node. */
int sgc_mgpu_init(int ndev, const int *devices);
int sgc_mgpu_attach(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                    int64_t n_rows, int64_t nnz, void *stream, int64_t *handle);
int sgc_mgpu_propagate(int64_t handle, const float *X0, int64_t ldx, float *out, int64_t ldo,
                       int64_t F, int32_t K, void *stream);
int sgc_mgpu_detach(int64_t handle);
int sgc_mgpu_finalize(void);

/* ---------------------------------------------------------------------------
 * Process warm-up (replaces nothing in the reference; a one-time cost the
 * reference's first torch.spmm pays inside torch).  The HIP runtime loads a
 * translation unit's code object on the first launch of any of its kernels;
 * sgc_warmup launches one empty kernel per unit selected in `units` on
 * `stream` (the current device) and waits for them, so those loads happen
 * here rather than inside the first sgc_precompute the caller times
 * (reddit.py:43,72-74).  Units: SGC_WARM_PROPAGATE = SpMM, ingest, plan,
 * sort, column groups, the exchanges' block copy; SGC_WARM_CLASSIFIER = linear, fused loss, cross-entropy;
 * SGC_WARM_LOADERS = normalisation, sub-graph.  Synchronous. */
enum { SGC_WARM_PROPAGATE = 1, SGC_WARM_CLASSIFIER = 2, SGC_WARM_LOADERS = 4 };
int sgc_warmup(uint32_t units, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SGC_AMD_H */
