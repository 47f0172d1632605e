// xent.hip -- fused SGC classifier training step on gfx950 (SURVEY.md 8(f)
// row 2): loss = mean_m CE(softmax(x_m W^T + b), y_m) and its gradients
// dW = G^T X / M, db = sum_m G_m / M with G = softmax - onehot -- what the
// reference's closure computes through nn.Linear + F.cross_entropy +
// backward (citation.py:47-49, reddit.py:55-58).
//
// Three launches, X read from HBM twice (the floor without keeping a
// 2.4 KB-per-row tile on chip between the two GEMMs):
//   A  xent_fwd_kernel    logits on fp32 MFMA (the linear_kernel mapping),
//                         row softmax / log-sum-exp across the 16-lane class
//                         groups (DPP shuffles), G -> global [M][C16] (fp32,
//                         padded classes 0), per-wave loss and dG column sums;
//   B  xent_dw_cols_kernel (up to 48 classes; round 6) dW partials over
//                         column blocks x row ranges on split-bf16 MFMA, or
//                         xent_dw_kernel: dW partial slabs, each block a
//                         contiguous run of rows reduced on fp32 MFMA
//                         (A = G^T straight from G's row-major layout,
//                         B = X rows, V-vector loads split over V MFMAs);
//   C  xent_reduce_kernel slabs -> dW, per-wave partials -> db and loss, in a
//                         fixed order (bitwise reproducible run to run).
#include "gemm_tile.h"
#include "split_bf16.h"

namespace sgc {


namespace {

__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
    return v;
}
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// ---- A: logits -> G, loss / dG partials ------------------------------------
template <int V, int NT, int NB>
__global__ __launch_bounds__(256) void xent_fwd_kernel(
    const float *__restrict__ X, int64_t ldx, const float *__restrict__ W,
    const float *__restrict__ b, const int64_t *__restrict__ labels, int M, int K, int C,
    float inv_m, float *__restrict__ G, int ldg, double *__restrict__ loss_part,
    float *__restrict__ db_part, float *__restrict__ logits, int64_t ldl) {
    __shared__ LdsTile<V, NT, NB> sm;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wave = blockIdx.x * 4 + w;
    const int i = lane & 15, g = lane >> 4;
    const int m_blk = blockIdx.x * kLdsBM;
    const int m0 = m_blk + w * 32;
    double wave_loss = 0.0;
    float dbc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) dbc[n] = 0.f;
    {
        f32x4 acc[2][NT];
        xwt_block_tile<V, NT, NB>(X, ldx, W, M, K, C, m_blk, sm, acc);
        float bias[NT];
        bool valid[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int c = n * 16 + i;
            valid[n] = c < C;
            bias[n] = (valid[n] && b) ? b[c] : 0.f;
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + t * 16 + g * 4 + r;
                const bool row_ok = m < M;  // uniform per (t, r, lane group)
                float z[NT];
                float mx = -INFINITY;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    z[n] = valid[n] ? acc[t][n][r] + bias[n] : -INFINITY;
                    mx = fmaxf(mx, z[n]);
                }
                mx = group16_max(mx);
                float se = 0.f;
#pragma unroll
                for (int n = 0; n < NT; ++n) se += valid[n] ? expf(z[n] - mx) : 0.f;
                se = group16_sum(se);
                const float lse = mx + logf(se);
                const int64_t y = row_ok ? labels[m] : -1;
                float zy = 0.f;
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    const int c = n * 16 + i;
                    const bool is_y = (c == y);
                    if (is_y) zy = z[n];
                    const float p = valid[n] ? expf(z[n] - lse) : 0.f;
                    const float gv = row_ok ? (p - (is_y ? 1.f : 0.f)) * inv_m : 0.f;
                    if (row_ok) {
                        G[(int64_t)m * ldg + c] = gv;
                        if (logits && valid[n]) logits[(int64_t)m * ldl + c] = z[n];
                    }
                    dbc[n] += gv;
                }
                zy = group16_sum(zy);  // exactly one lane of the group holds z_y
                if (row_ok && i == 0) wave_loss += (double)(lse - zy);
            }
    }
    // per-wave partials: loss (lanes i==0 of each group), dG column sums
    double l = wave_loss;
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (lane == 0) loss_part[wave] = l;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        float s = dbc[n];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (g == 0) db_part[(int64_t)wave * ldg + n * 16 + i] = s;
    }
}

#ifndef SGC_DW_SLABS
#define SGC_DW_SLABS 512
#endif
// dW partial slabs (workgroups of xent_dw_kernel) at most: each writes a
// C16 x K partial that the reduction reads back.  512 measured best at the
// Reddit-train shape: backward 0.142 ms vs 0.170 (256) and 0.191 (1024),
// profiles/r05/bwd_slabs_ab.log.
constexpr int64_t kDwSlabs = SGC_DW_SLABS;

// ---- B: dW partial slabs -----------------------------------------------------
constexpr int kDwDepth = 4;  // 4-row steps of G and X in flight per wave

// Host-side precondition of xent_dw_kernel's buffer offsets.
// (Both slab kernels load past the slab's last step -- up to 64 rows -- and
// read 0 there through the descriptors' ranges; the offsets must still fit.)
inline bool dw_slab_fits(int64_t rows_per, int64_t ldx, int64_t ldg) {
    return (rows_per + 64) * std::max(ldx, ldg) * 4 < (int64_t(1) << 31);
}

// Block blk reduces rows [blk*rows_per, ...) into slab[blk][C16][K].  Wave w
// owns the K column groups {w, w+4, ...} of 16*V columns each.  MFMA k-step =
// 4 rows: A[i=class][k=row] = G[row][class] (lane l: G[r0+(l>>4)][n*16+(l&15)]),
// B[k=row][j] = X[r0+(l>>4)][c0 + (l&15)*V + v] for MFMA v.
// Classes >= C read as 0 (G may be a caller's [M][C] gradient, ldg = C).
// db_slab (nullable): wave 0's first column group also sums its block's G
// rows per class (lane groups in row order, then across them) into
// db_slab[blk][C16] -- db = sum_m G_m from the same loads, in a fixed order.
template <int V, int NT, int CT>
__global__ __launch_bounds__(256) void xent_dw_kernel(const float *__restrict__ X, int64_t ldx,
                                                     const float *__restrict__ G, int ldg, int M,
                                                     int K, int C, int rows_per,
                                                     float *__restrict__ slab,
                                                     float *__restrict__ db_slab) {
    using VT = typename Vec<V>::T;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int r_begin = blockIdx.x * rows_per;
    const int r_end = min(M, r_begin + rows_per);
    const int group_cols = 16 * V;
    const int n_groups = (K + group_cols - 1) / group_cols;
    float *out = slab + (int64_t)blockIdx.x * (NT * 16) * K;
    for (int gb = w; gb < n_groups; gb += 4 * CT) {
        f32x4 acc[NT][CT][V];
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int v = 0; v < V; ++v) acc[n][ct][v] = f32x4{0.f, 0.f, 0.f, 0.f};
        // groups gb, gb+4, ...: how many exist (the last pass of some waves
        // has fewer than CT; round 5 ran their MFMAs anyway, 14 % of them)
        const int n_ct = min(CT, (n_groups - gb + 3) / 4);
        int coff[CT];
        bool cok[CT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const int c = (gb + ct * 4) * group_cols + i * V;
            cok[ct] = c < K;
            coff[ct] = cok[ct] ? c : 0;
        }
        // Buffer loads (round 4): one descriptor for the block's rows of X and
        // one for its rows of G, each lane's byte offset computed once and the
        // step's row offset a scalar, so a load costs one add.  Rows past
        // r_end lie outside both descriptors (zeros: the ragged last step
        // needs no code of its own) and so do classes >= C.  Columns past K
        // read column 0 (finite) and are never stored.
        const int n_rows = max(0, r_end - r_begin);  // 0: an empty trailing block
        const auto xdsc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(X + (int64_t)r_begin * ldx), 0,
            n_rows ? (int)(((int64_t)(n_rows - 1) * ldx + K) * 4) : 0, 0x00020000);
        const auto gdsc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(G + (int64_t)r_begin * ldg), 0,
            n_rows ? (int)(((int64_t)(n_rows - 1) * ldg + C) * 4) : 0, 0x00020000);
        uint32_t xo[CT], go[NT];
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) xo[ct] = (uint32_t)(g * ldx + coff[ct]) * 4u;
#pragma unroll
        for (int n = 0; n < NT; ++n)
            go[n] = (n * 16 + i < C) ? (uint32_t)(g * ldg + n * 16 + i) * 4u : kOffOOB;
        const bool sum_db = db_slab && gb == 0;  // wave 0, first column group: every row once
        float dba[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) dba[n] = 0.f;
        auto load = [&](int step, float (&gd)[NT], VT (&xd)[CT]) {
            const uint32_t rx = (uint32_t)(4 * step) * (uint32_t)ldx * 4u;
            const uint32_t rg = (uint32_t)(4 * step) * (uint32_t)ldg * 4u;
#pragma unroll
            for (int n = 0; n < NT; ++n)
                gd[n] = __builtin_bit_cast(float,
                                           __builtin_amdgcn_raw_buffer_load_b32(gdsc, go[n] + rg, 0, 0));
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) xd[ct] = buffer_load_vec<V>(xdsc, xo[ct] + rx);
        };
        auto mma = [&](const float (&gd)[NT], const VT (&xd)[CT]) {
            if (sum_db) {
#pragma unroll
                for (int n = 0; n < NT; ++n) dba[n] += gd[n];
            }
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                if (ct >= n_ct) break;  // wave-uniform: a group past K issues no MFMAs
#pragma unroll
                for (int v = 0; v < V; ++v)
#pragma unroll
                    for (int n = 0; n < NT; ++n)
                        acc[n][ct][v] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            gd[n], lane_elem<V>(xd[ct], v), acc[n][ct][v], 0, 0, 0);
            }
        };
        // kDwDepth 4-row steps in flight (a ring of register buffers): the
        // round-1 loop kept two and its waves sat 56 % of their cycles on
        // s_waitcnt (profiles/r04/pmc_cls/sq.summary)
        const int n_steps = (n_rows + 3) / 4;
        float gr[kDwDepth][NT];
        VT xr[kDwDepth][CT];
        // Every load is issued on every path (steps past the slab read 0
        // through the descriptors' ranges, dw_slab_fits covers their
        // offsets): a load under a branch made hipcc drain the whole ring
        // (vmcnt(0)) at each step, so the prefetch never overlapped the MFMAs
        // (round 6, profiles/r06/s5: MFMA-busy 51 % with the rest waiting).
#pragma unroll
        for (int d = 0; d < kDwDepth; ++d) load(d, gr[d], xr[d]);
        int s0 = 0;
        for (; s0 + kDwDepth <= n_steps; s0 += kDwDepth) {
#pragma unroll
            for (int d = 0; d < kDwDepth; ++d) {
                mma(gr[d], xr[d]);
                load(s0 + d + kDwDepth, gr[d], xr[d]);
            }
        }
#pragma unroll
        for (int d = 0; d < kDwDepth; ++d)  // the last n_steps % kDwDepth steps, already loaded
            if (s0 + d < n_steps) mma(gr[d], xr[d]);
        if (sum_db) {
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                float v = dba[n];
                v += __shfl_xor(v, 16, 64);
                v += __shfl_xor(v, 32, 64);
                if (g == 0) db_slab[(int64_t)blockIdx.x * (NT * 16) + n * 16 + i] = v;
            }
        }
        // D[class = 4*(l>>4)+q][j = l&15] of MFMA (n, ct, v) -> column c(j) + v
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const int c = (gb + ct * 4) * group_cols + i * V;
                if (!cok[ct]) continue;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int cls = n * 16 + g * 4 + q;
#pragma unroll
                    for (int v = 0; v < V; ++v) out[(int64_t)cls * K + c + v] = acc[n][ct][v][q];
                }
            }
    }
}

// ---- B': dW partial slabs on split-bf16 products (round 6) -----------------
// The same slab decomposition as xent_dw_kernel, with the fp32 MFMA
// (16x16x4: 8 instructions of 32 cycles per 32 rows of a 16 x 16 tile) replaced
// by the forward's exact three-piece bf16 split (split_bf16.h) on
// v_mfma_f32_16x16x32_bf16 (6 instructions of 16 cycles for the same tile):
// round 6's counters put xent_dw_kernel at 51 % MFMA-busy with the rest
// waiting on memory, i.e. the two costs in series (profiles/r06/s3/pmc_cls).
// The MFMA's k is the row: lane (g, i) needs rows 8g .. 8g+7 of one class /
// one column, which row-major loads give directly.
//   prologue  the block splits its slab's dY (G) once into LDS, in MFMA
//             A-operand order: [step][class tile n][piece][lane] x 16 B
//             (rows 8g .. 8g+7 of class 16n + i for lane (g, i)), and the
//             per-(step, lane) row sums for db;
//   passes    wave w takes the 32-column groups w, w+4, ...: lane (g, i) of
//             load t reads X[row 8g + t][c0 + 2i, c0 + 2i + 1] (8 B; column
//             2i feeds N-tile "even", 2i + 1 N-tile "odd": no lane exchange),
//             splits its 16 values, and runs 3 x 2 x 6 MFMAs against the LDS
//             pieces per 32 rows, the next step's X loads in flight.
// No transpose, one split of dY per slab (round 6's first form split it on
// every pass: 25 M VALU, slower than fp32).
// Measured (Reddit-train shape, rocprofv3 kernel means, profiles/r06/s8*):
// 107 us against the fp32 slabs' 112-115 us, but 681 slabs of 224 rows make
// the reduction 19.6 us against 16.3 (512 slabs): 127 vs 131 us in all, within
// run-to-run spread, so it stays opt-in (sgc_set_tuning("backward_kernel", 2)).
// Not kept: 16-B lanes over 64-column groups (115 us), 320-row slabs in two
// LDS phases (126 us), 160 / 128-row slabs (115 / 121 us + 28 / 35 us of
// reduction), a register cap for two workgroups per CU (spills: 256 us).
// The counters (profiles/r06/s6) put it at 58 % issue-stalled with MFMA busy
// 21 us of the 107: neither the MFMA nor the X stream (3.4 TB/s) bounds it.  Products hh go to accH, the five
// small ones to accL (as the forward kernel); dW = accH + accL per slab.
// Rows past the slab and classes >= C read 0 through the descriptors.
constexpr int kDwSplitRows = 224;  // slab rows (7 steps): 7 x 3 x 3 KB of LDS pieces
template <int NT>
struct DwSplitLds {
    u32x4 gp[kDwSplitRows / 32][NT][3][64];
    float dbp[kDwSplitRows / 32][NT][4][16];
};

template <int NT>
__global__ __launch_bounds__(256) void xent_dw_split_kernel(
    const float *__restrict__ X, int64_t ldx, const float *__restrict__ G, int ldg, int M, int K,
    int C, int rows_per, float *__restrict__ slab, float *__restrict__ db_slab) {
    __shared__ DwSplitLds<NT> sm;
    constexpr int kSteps = kDwSplitRows / 32;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int r_begin = blockIdx.x * rows_per;
    const int r_end = min(M, r_begin + rows_per);
    const int n_rows = max(0, r_end - r_begin);
    const int n_groups = (K + 31) / 32;
    const int n_steps = min(kSteps, (n_rows + 31) / 32);
    float *out = slab + (int64_t)blockIdx.x * (NT * 16) * K;
    const auto xdsc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(X + (int64_t)r_begin * ldx), 0,
        n_rows ? (int)(((int64_t)(n_rows - 1) * ldx + K) * 4) : 0, 0x00020000);
    const auto gdsc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(G + (int64_t)r_begin * ldg), 0,
        n_rows ? (int)(((int64_t)(n_rows - 1) * ldg + C) * 4) : 0, 0x00020000);
    // first pass's column group and its first X step: in flight under the prologue
    Vec<2>::T xv[2][8];
    auto xoff = [&](int gb) {
        const int c = gb * 32 + 2 * i;  // K is even: both columns in or out
        return (gb < n_groups && c < K) ? (uint32_t)(8 * g * ldx + c) * 4u : kOffOOB;
    };
    auto load_x = [&](int st, uint32_t xo, Vec<2>::T (&xd)[8]) {
#pragma unroll
        for (int t = 0; t < 8; ++t)
            xd[t] = buffer_load_vec<2>(xdsc, xo + (uint32_t)(32 * st + t) * (uint32_t)ldx * 4u);
    };
    uint32_t xo = xoff(w);
    load_x(0, xo, xv[0]);
    // prologue: item (step, tile, lane') -> pieces of rows 8g'..8g'+7, class 16n + i'
    for (int item = threadIdx.x; item < kSteps * NT * 64; item += 256) {
        const int st = item / (NT * 64), rem = item - st * NT * 64;
        const int n = rem >> 6, l = rem & 63, gi = l >> 4, ii = l & 15;
        const uint32_t go = (n * 16 + ii < C) ? (uint32_t)((32 * st + 8 * gi) * ldg + n * 16 + ii) * 4u
                                              : kOffOOB;
        float v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t)
            v[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                 gdsc, go + (uint32_t)t * (uint32_t)ldg * 4u, 0, 0));
        u32x4 ph, pm, pl;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t h, m, lo;
            split3(v[2 * q], v[2 * q + 1], h, m, lo);
            ph[q] = h;
            pm[q] = m;
            pl[q] = lo;
        }
        sm.gp[st][n][0][l] = ph;
        sm.gp[st][n][1][l] = pm;
        sm.gp[st][n][2][l] = pl;
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) sum += v[t];
        sm.dbp[st][n][gi][ii] = sum;
    }
    __syncthreads();
    if (db_slab && threadIdx.x < NT * 16) {  // db: steps, then lane groups, in order
        const int n = threadIdx.x >> 4, ii = threadIdx.x & 15;
        float sum = 0.f;
        for (int st = 0; st < kSteps; ++st)
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) sum += sm.dbp[st][n][gi][ii];
        db_slab[(int64_t)blockIdx.x * (NT * 16) + n * 16 + ii] = sum;
    }
    for (int gb = w; gb < n_groups; gb += 4) {
        f32x4 accH[NT][2], accL[NT][2];
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                accH[n][e] = f32x4{0.f, 0.f, 0.f, 0.f};
                accL[n][e] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        const uint32_t xo_next = xoff(gb + 4);
        auto step = [&](int st, const Vec<2>::T (&xd)[8]) {
            u32x4 gp[NT][3];
#pragma unroll
            for (int n = 0; n < NT; ++n)
#pragma unroll
                for (int p = 0; p < 3; ++p) gp[n][p] = sm.gp[st][n][p][lane];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                u32x4 xp[3];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t h, m, lo;
                    split3(xd[2 * q][e], xd[2 * q + 1][e], h, m, lo);
                    xp[0][q] = h;
                    xp[1][q] = m;
                    xp[2][q] = lo;
                }
                auto A = [&](int n, int p) { return __builtin_bit_cast(bf16x8_t, gp[n][p]); };
                auto B = [&](int p) { return __builtin_bit_cast(bf16x8_t, xp[p]); };
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    accH[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 0), B(0), accH[n][e], 0, 0, 0);
                    accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 0), B(1), accL[n][e], 0, 0, 0);
                    accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 1), B(0), accL[n][e], 0, 0, 0);
                    accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 0), B(2), accL[n][e], 0, 0, 0);
                    accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 2), B(0), accL[n][e], 0, 0, 0);
                    accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 1), B(1), accL[n][e], 0, 0, 0);
                }
            }
        };
        // steps in pairs on the two register sets; every load is issued on every
        // path (past the slab / past K: 0), the last one already the next
        // pass's first step, so hipcc's counted waits stay partial
#pragma unroll
        for (int st = 0; st < kSteps; st += 2) {
            if (st + 1 < kSteps) {
                load_x(st + 1, xo, xv[1]);
                if (st < n_steps) step(st, xv[0]);
                if (st + 2 < kSteps)
                    load_x(st + 2, xo, xv[0]);
                else
                    load_x(0, xo_next, xv[0]);
                if (st + 1 < n_steps) step(st + 1, xv[1]);
            } else {
                const Vec<2>::T(&cur)[8] = xv[0];
                Vec<2>::T keep[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) keep[t] = cur[t];
                load_x(0, xo_next, xv[0]);
                if (st < n_steps) step(st, keep);
            }
        }
        // D[class = 4*(l>>4)+q][j = l&15] of tile (n, e) -> column gb*32 + 2j + e
        const int c = gb * 32 + 2 * i;
        if (c < K) {
#pragma unroll
            for (int n = 0; n < NT; ++n)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int cls = n * 16 + g * 4 + q;
                    Vec<2>::T v2;
                    v2[0] = accH[n][0][q] + accL[n][0][q];
                    v2[1] = accH[n][1][q] + accL[n][1][q];
                    *reinterpret_cast<Vec<2>::T *>(out + (int64_t)cls * K + c) = v2;
                }
        }
        xo = xo_next;
    }
}

// NT consecutive floats at byte offset off (one 4-, 8- or 12-B buffer load;
// past the range: 0 per dword)
template <int NT>
__device__ __forceinline__ void buffer_load_floats(__amdgpu_buffer_rsrc_t r, uint32_t off,
                                                   float (&v)[NT]) {
    static_assert(NT >= 1 && NT <= 3, "1-3 floats");
    if constexpr (NT == 3) {
        typedef float f3 __attribute__((ext_vector_type(3)));
        const f3 x = __builtin_bit_cast(f3, __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 0));
        v[0] = x[0];
        v[1] = x[1];
        v[2] = x[2];
    } else if constexpr (NT == 2) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 x = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
        v[0] = x[0];
        v[1] = x[1];
    } else {
        v[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
    }
}

// ---- B'': dW on split-bf16 products over column blocks (round 6) -----------
// What B and B' spend besides the stream: a C16 x K partial per 224-300-row
// slab -- 512-681 partials, 59-79 MB written and read back by the reduction,
// a fifth of the algorithmic bytes -- and for B' 1.33 rounds of blocks.  Here a
// block owns a 64-column block cb of X and a row "range" r (R ranges: R x
// ceil(K / 64) blocks, one round at two blocks per CU).  Range r is the
// 32-row steps r, r + R, r + 2R, ... and the block's wave w takes every fourth
// of them, so at any moment the grid reads X inside a window of ~4R steps
// (contiguous ranges, 48 separate runs: loads alone 78 vs 76 us, whole kernel
// 1-2 us slower, profiles/r06/s18); a step's own descriptors bound it (rows
// past M read 0).  Per step lane (g, i) reads
//   dY rows 32s + 8g + t (t < 8), classes NT i .. NT i + NT - 1 (one 4-, 8- or
//      12-B load per row): row i of class tile n is class NT i + n, so a
//      lane's classes are adjacent in dY's row (8 loads a step, not 8 NT),
//      the A operands of the NT tiles, and
//   X rows 32s + 8g + t, columns c0 + 4i .. c0 + 4i + 3 (16-B loads; 4 rows
//      x 256 B per instruction): the B operands of N-tiles e = 0..3 (column
//      c0 + 4i + e), no lane exchange,
// splits both into three bf16 pieces (split_bf16.h) and runs NT x 4 x 6
// v_mfma_f32_16x16x32_bf16, the next step's loads in flight.  The waves'
// accumulators are summed in LDS in wave order and the block stores its 64
// columns of partial r: R partials in all (48 at the Reddit-train shape:
// 4.7 MB).  dY is read by each column block of a range; block b runs on XCD
// b % 8, and the blocks of range r are numbered so b % 8 == r % 8: a range's
// ten dY reads share one L2.  Columns past K read whatever lies there (the
// next row, or 0 past the step) and are never stored: column j of dW
// depends on column j of X only.
#ifndef SGC_DW_COL_RANGES
#define SGC_DW_COL_RANGES 48
#endif
constexpr int kDwColRanges = SGC_DW_COL_RANGES;  // row ranges (a multiple of 8: the XCD numbering)
constexpr int kDwColWidth = 64;   // columns per block

template <int NT>
__global__ __launch_bounds__(256) void xent_dw_cols_kernel(
    const float *__restrict__ X, int64_t ldx, const float *__restrict__ G, int ldg, int M, int K,
    int C, int n_cblk, int R, float *__restrict__ slab, float *__restrict__ db_slab) {
    __shared__ f32x4 red[4][NT][4][64];  // [wave][class tile][q][lane] -> N-tiles e = 0..3
    __shared__ float dbr[4][NT * 16];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform loop bounds
    const int i = lane & 15, g = lane >> 4;
    const int q8 = (int)blockIdx.x >> 3;
    const int cb = q8 % n_cblk, r = (q8 / n_cblk) * 8 + ((int)blockIdx.x & 7);
    if (r >= R) return;  // (uniform per block: no barrier reached)
    const int S = (M + 31) >> 5;
    const int c0 = cb * kDwColWidth;
    const uint32_t xpitch = (uint32_t)ldx * 4u, gpitch = (uint32_t)ldg * 4u;
    // a lane whose four columns all lie past K reads nothing (the last block's
    // lanes would otherwise read the next row's first columns)
    const uint32_t xlane = c0 + 4 * i < K ? (uint32_t)(8 * g * ldx + c0 + 4 * i) * 4u : kOffOOB;
    // classes NT i + n; a lane whose first class is past C reads nothing (a
    // partly valid lane reads classes past C from the next row or as 0: they
    // reach only rows of dW past C, never stored)
    const uint32_t glane = NT * i < C ? (uint32_t)(8 * g * ldg + NT * i) * 4u : kOffOOB;
    f32x4 xr[8];
    float gr[8][NT];
    // range r's steps are r, r + R, r + 2R, ... and wave w takes every fourth
    // of them: at any moment the whole grid reads inside a window of ~4R
    // steps of X, not R separate runs; a step's own descriptors (rows past M,
    // and steps past the last, read 0)
    const int w_a = w, w_b = (S - r + R - 1) / R, w_step = 4;
    auto load = [&](int j) {
        const int s = r + R * j;
        const int rows = s < S ? min(32, M - 32 * s) : 0;
        const int64_t row0 = s < S ? 32 * (int64_t)s : 0;
        const auto xd = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(X + row0 * ldx), 0, rows ? (int)(((int64_t)(rows - 1) * ldx + K) * 4) : 0,
            0x00020000);
        const auto gd = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(G + row0 * ldg), 0, rows ? (int)(((int64_t)(rows - 1) * ldg + C) * 4) : 0,
            0x00020000);
        // (the lane offsets opaque per step: hoisted, the 16 row offsets would
        // hold 16 VGPRs for the whole loop and cost the second wave per SIMD)
        uint32_t xl = xlane, gl = glane;
        asm volatile("" : "+v"(xl), "+v"(gl));
#pragma unroll
        for (int t = 0; t < 8; ++t)
            xr[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  xd, xl + (uint32_t)t * xpitch, 0, 0));
#pragma unroll
        for (int t = 0; t < 8; ++t) buffer_load_floats<NT>(gd, gl + (uint32_t)t * gpitch, gr[t]);
    };
    // hh products in accH, the five small ones in accL (as the forward)
    f32x4 accH[NT][4], accL[NT][4];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            accH[n][e] = f32x4{0.f, 0.f, 0.f, 0.f};
            accL[n][e] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    const bool sum_db = db_slab && cb == 0;  // column block 0 also sums dY's rows
    float dba[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) dba[n] = 0.f;
    load(w_a);
    for (int st = w_a; st < w_b; st += w_step) {
        u32x4 ga[NT][3], xb[4][3];
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t h, m, lo;
                split3(gr[2 * q][n], gr[2 * q + 1][n], h, m, lo);
                ga[n][0][q] = h;
                ga[n][1][q] = m;
                ga[n][2][q] = lo;
            }
        if (sum_db) {
#pragma unroll
            for (int n = 0; n < NT; ++n)
#pragma unroll
                for (int t = 0; t < 8; ++t) dba[n] += gr[t][n];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t h, m, lo;
                split3(xr[2 * q][e], xr[2 * q + 1][e], h, m, lo);
                xb[e][0][q] = h;
                xb[e][1][q] = m;
                xb[e][2][q] = lo;
            }
        load(st + w_step);
        // the next step's loads go out before this step's MFMAs (the
        // scheduler otherwise interleaves the splits with the MFMAs and
        // issues the loads two thirds of the way through them)
        __builtin_amdgcn_sched_barrier(0);
#if defined(SGC_DW_COLS_DIAG) && SGC_DW_COLS_DIAG == 1  // measurement: loads only
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) accH[0][e][t & 3] += xr[t][e] + gr[t][e % NT];
        continue;
#elif defined(SGC_DW_COLS_DIAG) && SGC_DW_COLS_DIAG == 2  // measurement: loads + splits
        uint32_t fold = 0;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#pragma unroll
                for (int e = 0; e < 4; ++e) fold ^= xb[e][p][q];
#pragma unroll
                for (int n = 0; n < NT; ++n) fold ^= ga[n][p][q];
            }
        accH[0][0][0] += __uint_as_float(fold & 0x807fffffu);
        continue;
#endif
        auto A = [&](int n, int p) { return __builtin_bit_cast(bf16x8_t, ga[n][p]); };
        auto B = [&](int e, int p) { return __builtin_bit_cast(bf16x8_t, xb[e][p]); };
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                accH[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 0), B(e, 0), accH[n][e], 0, 0, 0);
                accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 0), B(e, 1), accL[n][e], 0, 0, 0);
                accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 1), B(e, 0), accL[n][e], 0, 0, 0);
                accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 0), B(e, 2), accL[n][e], 0, 0, 0);
                accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 2), B(e, 0), accL[n][e], 0, 0, 0);
                accL[n][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A(n, 1), B(e, 1), accL[n][e], 0, 0, 0);
            }
    }
    // D[row 4g + q][j = i] of tile (n, e) -> class NT (4g + q) + n, column c0 + 4i + e
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            red[w][n][q][lane] = f32x4{accH[n][0][q] + accL[n][0][q], accH[n][1][q] + accL[n][1][q],
                                       accH[n][2][q] + accL[n][2][q], accH[n][3][q] + accL[n][3][q]};
    if (sum_db) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            float v = dba[n];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            if (g == 0) dbr[w][NT * i + n] = v;
        }
    }
    __syncthreads();
    // the block's partial: classes < C x its columns < K, the waves in order;
    // thread (cls = NT (4 gg + q) + n, col): red[.][n][q][16 gg + ii][e] is
    // float 64 gg + col of row (n, q)
    const int col = threadIdx.x & 63;
    const float *rf = reinterpret_cast<const float *>(red);
    float *out = slab + (int64_t)r * (NT * 16) * K;
    if (c0 + col < K) {
        for (int cls = threadIdx.x >> 6; cls < C; cls += 4) {
            const int r4 = cls / NT, n = cls - r4 * NT, gg = r4 >> 2, q = r4 & 3;
            const int at = ((n * 4 + q) * 64) * 4 + 64 * gg + col;
            constexpr int wstride = NT * 4 * 64 * 4;
            out[(int64_t)cls * K + c0 + col] =
                ((rf[at] + rf[at + wstride]) + rf[at + 2 * wstride]) + rf[at + 3 * wstride];
        }
    }
    if (sum_db && (int)threadIdx.x < C)
        db_slab[(int64_t)r * (NT * 16) + threadIdx.x] =
            ((dbr[0][threadIdx.x] + dbr[1][threadIdx.x]) + dbr[2][threadIdx.x]) + dbr[3][threadIdx.x];
}

// ---- C: fixed-order reductions ----------------------------------------------
// dW: a block owns 64 consecutive elements; wave w sums slabs [w*n/4, (w+1)*n/4)
// in order (coalesced 256-B rows of each slab), then wave 0 adds the four
// partials in order.  Deterministic; ~n/4 loads in flight per lane.
__global__ __launch_bounds__(256) void xent_reduce_dw_kernel(const float *__restrict__ slab,
                                                             int n_slabs, int C, int K, int C16,
                                                             float *__restrict__ dW) {
    __shared__ float part[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t e = blockIdx.x * 64LL + lane;
    const int64_t total = (int64_t)C * K;
    const int j0 = (int)((int64_t)n_slabs * w / 4), j1 = (int)((int64_t)n_slabs * (w + 1) / 4);
    float s = 0.f;
    if (e < total) {
        const int64_t cls = e / K, k = e - cls * K;
        const float *p = slab + cls * K + k;
        const int64_t stride = (int64_t)C16 * K;
        int j = j0;
        for (; j + 8 <= j1; j += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(j + u) * stride];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; j < j1; ++j) s += p[(int64_t)j * stride];
    }
    part[w][lane] = s;
    __syncthreads();
    if (w == 0 && e < total) dW[e] = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
}

// dW as xent_reduce_dw_kernel, and in the same launch db: blocks past dW's
// (one per 64 classes) sum db_slab's column over the slabs, wave w a quarter
// of them in order, then the four partials in order -- the backward's two
// reductions in one launch (round 5 ran db as a second, 5.5 us launch).
__global__ __launch_bounds__(256) void xent_reduce_dw_db_kernel(
    const float *__restrict__ slab, int n_slabs, int C, int K, int C16, float *__restrict__ dW,
    const float *__restrict__ db_slab, float *__restrict__ db, int dw_blocks) {
    __shared__ float part[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j0 = (int)((int64_t)n_slabs * w / 4), j1 = (int)((int64_t)n_slabs * (w + 1) / 4);
    float s = 0.f;
    bool ok;
    int64_t e;
    if ((int)blockIdx.x < dw_blocks) {
        e = blockIdx.x * 64LL + lane;
        ok = e < (int64_t)C * K;
        if (ok) {
            const int64_t cls = e / K, k = e - cls * K;
            const float *p = slab + cls * K + k;
            const int64_t stride = (int64_t)C16 * K;
            // 16 loads in flight per batch (the column-block kernel's 48
            // partials: one batch per wave; a slot past j1 adds 0)
            for (int j = j0; j < j1; j += 16) {
                float v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = j + u < j1 ? p[(int64_t)(j + u) * stride] : 0.f;
#pragma unroll
                for (int u = 0; u < 16; ++u) s += v[u];
            }
        }
    } else {
        // db: one wave per class -- lane l sums slabs l, l + 64, ... (eight
        // loads in flight), then a fixed xor tree across the wave (round 6's
        // first form had one lane walk a quarter of the slabs: 49 us)
        const int cls = (blockIdx.x - dw_blocks) * 4 + w;
        if (cls < C) {
            const float *p = db_slab + cls;
            int j = lane;
            for (; j + 7 * 64 < n_slabs; j += 8 * 64) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(j + u * 64) * C16];
#pragma unroll
                for (int u = 0; u < 8; ++u) s += v[u];
            }
            for (; j < n_slabs; j += 64) s += p[(int64_t)j * C16];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
            if (lane == 0) db[cls] = s;
        }
        return;  // (uniform per block: no barrier below is reached)
    }
    part[w][lane] = s;
    __syncthreads();
    if (w == 0 && ok) dW[e] = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
}

// loss (double, block C) and db (block c < C): 256 threads per block, strided
// partial sums then a fixed-shape LDS tree -- deterministic.
__global__ __launch_bounds__(256) void xent_reduce_small_kernel(
    const double *__restrict__ loss_part, const float *__restrict__ db_part, int n_waves, int C,
    int ldg, double inv_m, float *__restrict__ loss, float *__restrict__ db) {
    __shared__ double red[256];
    const int t = threadIdx.x, c = blockIdx.x;
    if (c < C && !db) return;
    double s = 0.0;
    if (c == C) {
        for (int j = t; j < n_waves; j += 256) s += loss_part[j];
    } else {
        float f = 0.f;
        for (int j = t; j < n_waves; j += 256) f += db_part[(int64_t)j * ldg + c];
        s = f;
    }
    red[t] = s;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (t < h) red[t] += red[t + h];
        __syncthreads();
    }
    if (t == 0) {
        if (c == C)
            *loss = (float)(red[0] * inv_m);
        else
            db[c] = (float)red[0];
    }
}

template <int V, int NT>
hipError_t launch_fwd(const float *X, int64_t ldx, const float *W, const float *b,
                      const int64_t *labels, int M, int K, int C, float *G, int ldg,
                      double *loss_part, float *db_part, float *logits, int64_t ldl,
                      hipStream_t s) {
    const int blocks = (M + kLdsBM - 1) / kLdsBM;
    if (g_tile_buffers == 1)
        hipLaunchKernelGGL((xent_fwd_kernel<V, NT, 1>), dim3(blocks), dim3(256), 0, s, X, ldx, W,
                           b, labels, M, K, C, 1.0f / (float)M, G, ldg, loss_part, db_part, logits,
                           ldl);
    else
        hipLaunchKernelGGL((xent_fwd_kernel<V, NT, 2>), dim3(blocks), dim3(256), 0, s, X, ldx, W,
                           b, labels, M, K, C, 1.0f / (float)M, G, ldg, loss_part, db_part, logits,
                           ldl);
    return hipGetLastError();
}

template <int V, int NT>
hipError_t launch_dw(const float *X, int64_t ldx, const float *G, int ldg, int M, int K, int C,
                     int n_slabs, int rows_per, float *slab, float *db_slab, hipStream_t s) {
    constexpr int CT = (NT >= 3) ? 2 : 4;
    hipLaunchKernelGGL((xent_dw_kernel<V, NT, CT>), dim3(n_slabs), dim3(256), 0, s, X, ldx, G,
                       ldg, M, K, C, rows_per, slab, db_slab);
    return hipGetLastError();
}

template <int NT>
hipError_t launch_dw_split(const float *X, int64_t ldx, const float *G, int ldg, int M, int K,
                           int C, int n_slabs, int rows_per, float *slab, float *db_slab,
                           hipStream_t s) {
    hipLaunchKernelGGL((xent_dw_split_kernel<NT>), dim3(n_slabs), dim3(256), 0, s, X, ldx, G,
                       ldg, M, K, C, rows_per, slab, db_slab);
    return hipGetLastError();
}

// Row ranges of xent_dw_cols_kernel: kDwColRanges, fewer when M has fewer
// 32-row steps.
inline int dw_col_ranges(int64_t M) {
    return (int)std::min<int64_t>(kDwColRanges, std::max<int64_t>(1, (M + 31) / 32));
}

template <int NT>
hipError_t launch_dw_cols(const float *X, int64_t ldx, const float *G, int ldg, int M, int K,
                          int C, float *slab, float *db_slab, hipStream_t s) {
    const int R = dw_col_ranges(M);
    const int n_cblk = (K + kDwColWidth - 1) / kDwColWidth;
    const int blocks = n_cblk * ((R + 7) / 8) * 8;
    hipLaunchKernelGGL((xent_dw_cols_kernel<NT>), dim3(blocks), dim3(256), 0, s, X, ldx, G, ldg, M,
                       K, C, n_cblk, R, slab, db_slab);
    return hipGetLastError();
}

}  // namespace

// Backward kernel choice (sgc_set_tuning("backward_kernel")): 0 auto (the
// split-bf16 column blocks up to 48 classes, the fp32 MFMA slabs above), 1 the
// fp32 MFMA slabs, 2 the split-bf16 slabs where X gives 8-B lanes, 3 the
// split-bf16 column blocks (up to 48 classes).
int g_backward_kernel = 0;

static bool backward_split(int64_t K, int64_t ldx, const float *X) {
    return g_backward_kernel == 2 && K % 2 == 0 && ldx % 2 == 0 && (uintptr_t)X % 8 == 0;
}

static bool backward_cols(int64_t C) {
    return (g_backward_kernel == 0 || g_backward_kernel == 3) && C <= 48;
}

int64_t xent_workspace_bytes(int64_t M, int64_t K, int64_t C) {
    if (M <= 0 || K <= 0 || C <= 0) return 0;
    const int64_t C16 = (C + 15) / 16 * 16;
    const int64_t waves = (M + kLdsBM - 1) / kLdsBM * 4;
    // dW partials: the fp32 slabs' or the column blocks' row ranges
    const int64_t n_slabs = std::max<int64_t>(std::min<int64_t>(kDwSlabs, (M + 255) / 256),
                                              dw_col_ranges(M));
    auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
    return al(M * C16 * 4) + al(waves * 8) + al(waves * C16 * 4) + al(n_slabs * C16 * K * 4) + 512;
}

int linear_xent_f32(const float *X, int64_t ldx, const float *W, const float *b,
                    const int64_t *labels, int64_t M, int64_t K, int64_t C, float *loss,
                    float *dW, float *db, float *logits, int64_t ldl, void *ws, int64_t ws_bytes,
                    hipStream_t s) {
    SGC_REQUIRE(X && W && labels && loss && dW && ws, SGC_EINVAL, "linear_xent: null pointer");
    SGC_REQUIRE(M > 0 && K > 0 && C > 0 && C <= 64 && ldx >= K, SGC_EINVAL,
                "linear_xent: bad shape M=%lld K=%lld C=%lld (C <= 64)", (long long)M,
                (long long)K, (long long)C);
    SGC_REQUIRE(M < INT32_MAX && K < INT32_MAX, SGC_ERANGE, "linear_xent: too large");
    SGC_REQUIRE(!logits || ldl >= C, SGC_EINVAL, "linear_xent: ldl < C");
    SGC_REQUIRE(block_tile_fits(ldx, K, C), SGC_ERANGE,
                "linear_xent: ldx=%lld / K=%lld past the tile's 31-bit offsets", (long long)ldx,
                (long long)K);
    const int64_t need = xent_workspace_bytes(M, K, C);
    SGC_REQUIRE(ws_bytes >= need, SGC_ENOMEM, "linear_xent: workspace %lld < %lld",
                (long long)ws_bytes, (long long)need);
    const int NT = (int)((C + 15) / 16);
    const int C16 = NT * 16;
    const int waves = (int)((M + kLdsBM - 1) / kLdsBM * 4);
    const int n_slabs = (int)std::min<int64_t>(kDwSlabs, (M + 255) / 256);
    const int rows_per = (int)(((M + n_slabs - 1) / n_slabs + 3) / 4 * 4);
    SGC_REQUIRE(dw_slab_fits(rows_per, ldx, NT * 16), SGC_ERANGE,
                "classifier dW: %d rows x ldx %lld past the kernel's 31-bit offsets", rows_per,
                (long long)ldx);
    auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
    char *p = (char *)(((uintptr_t)ws + 255) & ~uintptr_t(255));
    float *G = (float *)p;
    p += al(M * C16 * 4);
    double *loss_part = (double *)p;
    p += al((int64_t)waves * 8);
    float *db_part = (float *)p;
    p += al((int64_t)waves * C16 * 4);
    float *slab = (float *)p;

    // dW on the split-bf16 column blocks up to 48 classes (as the backward)
    const bool cols = backward_cols(C) && dw_slab_fits(32, ldx, C16);
    const int n_parts = cols ? dw_col_ranges(M) : n_slabs;
    int V = 1;
    for (int v : {4, 2})
        if (K % v == 0 && ldx % v == 0 && (uintptr_t)X % (4 * v) == 0 && (uintptr_t)W % (4 * v) == 0) {
            V = v;
            break;
        }
    hipError_t e = hipSuccess;
#define SGC_XENT_DISPATCH(VV)                                                                    \
    switch (NT) {                                                                                \
        case 1: e = launch_fwd<VV, 1>(X, ldx, W, b, labels, (int)M, (int)K, (int)C, G, C16,      \
                                      loss_part, db_part, logits, ldl, s);                       \
            if (e == hipSuccess)                                                                 \
                e = cols ? launch_dw_cols<1>(X, ldx, G, C16, (int)M, (int)K, (int)C, slab, nullptr, s) \
                         : launch_dw<VV, 1>(X, ldx, G, C16, (int)M, (int)K, C16, n_slabs, rows_per,   \
                                              slab, nullptr, s);                                        \
            break;                                                                               \
        case 2: e = launch_fwd<VV, 2>(X, ldx, W, b, labels, (int)M, (int)K, (int)C, G, C16,      \
                                      loss_part, db_part, logits, ldl, s);                       \
            if (e == hipSuccess)                                                                 \
                e = cols ? launch_dw_cols<2>(X, ldx, G, C16, (int)M, (int)K, (int)C, slab, nullptr, s) \
                         : launch_dw<VV, 2>(X, ldx, G, C16, (int)M, (int)K, C16, n_slabs, rows_per,   \
                                              slab, nullptr, s);                                        \
            break;                                                                               \
        case 3: e = launch_fwd<VV, 3>(X, ldx, W, b, labels, (int)M, (int)K, (int)C, G, C16,      \
                                      loss_part, db_part, logits, ldl, s);                       \
            if (e == hipSuccess)                                                                 \
                e = cols ? launch_dw_cols<3>(X, ldx, G, C16, (int)M, (int)K, (int)C, slab, nullptr, s) \
                         : launch_dw<VV, 3>(X, ldx, G, C16, (int)M, (int)K, C16, n_slabs, rows_per,   \
                                              slab, nullptr, s);                                        \
            break;                                                                               \
        default: e = launch_fwd<VV, 4>(X, ldx, W, b, labels, (int)M, (int)K, (int)C, G, C16,     \
                                       loss_part, db_part, logits, ldl, s);                      \
            if (e == hipSuccess) e = launch_dw<VV, 4>(X, ldx, G, C16, (int)M, (int)K, C16,    \
                                                      n_slabs, rows_per, slab, nullptr, s);                        \
            break;                                                                               \
    }
    if (V == 4) {
        SGC_XENT_DISPATCH(4)
    } else if (V == 2) {
        SGC_XENT_DISPATCH(2)
    } else {
        SGC_XENT_DISPATCH(1)
    }
#undef SGC_XENT_DISPATCH
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "linear_xent launch failed: %s", hipGetErrorString(e));
    const int64_t ck = C * K;
    hipLaunchKernelGGL(xent_reduce_dw_kernel, dim3((unsigned)((ck + 63) / 64)), dim3(256), 0, s,
                       slab, n_parts, (int)C, (int)K, C16, dW);
    SGC_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(xent_reduce_small_kernel, dim3((unsigned)C + 1), dim3(256), 0, s, loss_part, db_part,
                       waves, (int)C, C16, 1.0 / (double)M, loss, db);
    SGC_HIP_CHECK(hipGetLastError());
    return SGC_OK;
}

// Backward of the classifier forward Y = X W^T + b (reference models.py:18,
// what autograd runs after F.cross_entropy(model(x), y).backward() in the
// closures of citation.py:47-49 / reddit.py:55-58): dW = dY^T X and
// db = sum_m dY_m from ONE read of X -- the dW slab kernel of the fused step
// with the caller's dY as G (classes past C masked) and the db column sums
// taken from the same G loads, then the two fixed-order reductions.
int64_t linear_backward_workspace_bytes(int64_t M, int64_t K, int64_t C) {
    if (M <= 0 || K <= 0 || C <= 0) return 0;
    const int64_t C16 = (C + 15) / 16 * 16;
    // the larger of the two kernels' slab counts (fp32: <= kDwSlabs slabs;
    // split-bf16: kDwSplitRows rows each)
    const int64_t n_slabs = std::max<int64_t>(
        std::max<int64_t>(std::min<int64_t>(kDwSlabs, (M + 255) / 256),
                          (M + kDwSplitRows - 1) / kDwSplitRows),
        dw_col_ranges(M));
    auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
    return al(n_slabs * C16 * K * 4) + al(n_slabs * C16 * 4) + 512;
}

int linear_backward_f32(const float *X, int64_t ldx, const float *dY, int64_t ldd, int64_t M,
                        int64_t K, int64_t C, float *dW, float *db, void *ws, int64_t ws_bytes,
                        hipStream_t s) {
    SGC_REQUIRE(X && dY && dW && ws, SGC_EINVAL, "linear_backward: null pointer");
    SGC_REQUIRE(M > 0 && K > 0 && C > 0 && C <= 64 && ldx >= K && ldd >= C, SGC_EINVAL,
                "linear_backward: bad shape M=%lld K=%lld C=%lld (C <= 64)", (long long)M,
                (long long)K, (long long)C);
    SGC_REQUIRE(M < INT32_MAX && K < INT32_MAX && ldd < INT32_MAX, SGC_ERANGE,
                "linear_backward: too large");
    const int64_t need = linear_backward_workspace_bytes(M, K, C);
    SGC_REQUIRE(ws_bytes >= need, SGC_ENOMEM, "linear_backward: workspace %lld < %lld",
                (long long)ws_bytes, (long long)need);
    const int NT = (int)((C + 15) / 16);
    const int C16 = NT * 16;
    const int max_slabs = (int)std::min<int64_t>(kDwSlabs, (M + 255) / 256);
    // the split-bf16 slabs need 8-B lanes of X (K, ldx even, X 8-B aligned)
    const bool split = backward_split(K, ldx, X);
    const int64_t per = (M + max_slabs - 1) / max_slabs;
    const int rows_per = (int)(split ? kDwSplitRows : (per + 3) / 4 * 4);
    const int n_slabs = (int)((M + rows_per - 1) / rows_per);  // workspace: see above
    SGC_REQUIRE(dw_slab_fits(rows_per, ldx, ldd), SGC_ERANGE,
                "classifier dW: %d rows x ldx %lld past the kernel's 31-bit offsets", rows_per,
                (long long)ldx);
    auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
    char *p = (char *)(((uintptr_t)ws + 255) & ~uintptr_t(255));
    float *slab = (float *)p;
    p += al((int64_t)std::max<int64_t>(
                std::max<int64_t>(max_slabs, (M + kDwSplitRows - 1) / kDwSplitRows),
                dw_col_ranges(M)) *
            C16 * K * 4);
    float *db_slab = db ? (float *)p : nullptr;
    int V = 1;
    for (int v : {4, 2})
        if (K % v == 0 && ldx % v == 0 && (uintptr_t)X % (4 * v) == 0) {
            V = v;
            break;
        }
    hipError_t e = hipSuccess;
    const bool cols = backward_cols(C);
    int n_parts = n_slabs;
    if (cols) {
        // a step's 32 rows are one descriptor's range
        SGC_REQUIRE(dw_slab_fits(32, ldx, ldd), SGC_ERANGE,
                    "classifier dW: 32 rows x ldx %lld past the kernel's 31-bit offsets",
                    (long long)ldx);
        n_parts = dw_col_ranges(M);
        switch (NT) {
            case 1: e = launch_dw_cols<1>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, slab,
                                          db_slab, s); break;
            case 2: e = launch_dw_cols<2>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, slab,
                                          db_slab, s); break;
            default: e = launch_dw_cols<3>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, slab,
                                           db_slab, s); break;
        }
    } else if (split) {
        switch (NT) {
            case 1: e = launch_dw_split<1>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, n_slabs,
                                           rows_per, slab, db_slab, s); break;
            case 2: e = launch_dw_split<2>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, n_slabs,
                                           rows_per, slab, db_slab, s); break;
            case 3: e = launch_dw_split<3>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, n_slabs,
                                           rows_per, slab, db_slab, s); break;
            default: e = launch_dw_split<4>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, n_slabs,
                                            rows_per, slab, db_slab, s); break;
        }
    } else {
#define SGC_BWD_DISPATCH(VV)                                                                     \
    switch (NT) {                                                                                \
        case 1: e = launch_dw<VV, 1>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, n_slabs,      \
                                     rows_per, slab, db_slab, s); break;                         \
        case 2: e = launch_dw<VV, 2>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, n_slabs,      \
                                     rows_per, slab, db_slab, s); break;                         \
        case 3: e = launch_dw<VV, 3>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, n_slabs,      \
                                     rows_per, slab, db_slab, s); break;                         \
        default: e = launch_dw<VV, 4>(X, ldx, dY, (int)ldd, (int)M, (int)K, (int)C, n_slabs,     \
                                      rows_per, slab, db_slab, s); break;                        \
    }
        if (V == 4) {
            SGC_BWD_DISPATCH(4)
        } else if (V == 2) {
            SGC_BWD_DISPATCH(2)
        } else {
            SGC_BWD_DISPATCH(1)
        }
#undef SGC_BWD_DISPATCH
    }
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "linear_backward launch failed: %s",
                hipGetErrorString(e));
    // dW and db in one launch (fixed-order sums over the slabs)
    const int dw_blocks = (int)((C * K + 63) / 64);
    const int db_blocks = db ? (int)((C + 3) / 4) : 0;  // a wave per class
    hipLaunchKernelGGL(xent_reduce_dw_db_kernel, dim3((unsigned)(dw_blocks + db_blocks)),
                       dim3(256), 0, s, slab, n_parts, (int)C, (int)K, C16, dW, db_slab, db,
                       dw_blocks);
    SGC_HIP_CHECK(hipGetLastError());
    return SGC_OK;
}

const char *linear_backward_kernel_name(int64_t M, int64_t K, int64_t ldx, int64_t C,
                                        const float *X) {
    if (M <= 0 || K <= 0 || C <= 0 || C > 64 || ldx < K) return "none";
    const bool split = backward_split(K, ldx, X);
    if (backward_cols(C))
        return "xent_dw_cols_kernel (split-bf16 column blocks, v_mfma_f32_16x16x32_bf16 x 6 products)";
    return split ? "xent_dw_split_kernel (split-bf16 slabs, v_mfma_f32_16x16x32_bf16 x 6 products)"
                 : "xent_dw_kernel (fp32 slabs, v_mfma_f32_16x16x4_f32)";
}

SGC_WARM_UNIT(warm_xent)

}  // namespace sgc
