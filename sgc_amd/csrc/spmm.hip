// spmm.hip -- CSR SpMM  Y = S[rows] . X  for gfx950 (MI355X), bit-exact with
// the reference CPU path (torch.spmm at /root/reference/utils.py:95).
//
// Numerical contract (pinned by tests/golden): every output
// element is ONE sequential fp32 FMA chain over its row's nonzeros in CSR
// order, starting from +0.0f.  So a lane owns features and walks the row's
// nonzeros in order; no (row, feature) sum is ever split across lanes or
// waves.  The one split is across launches, in order: with
// SGC_SPMM_ACCUMULATE a launch over column block g of S continues each chain
// from the fp32 value block g-1's launch stored (an exact round trip), so the
// passes over blocks 0, 1, ... of a row's CSR-ordered nonzeros are one chain.
//
// Mapping (one wavefront = 64 lanes per work item):
//   * features are cut into slices of 64*C*V floats (grid y); each slice is
//     a complete pass over S, so the live part of X is N x slice floats (see
//     the kernel comment: Infinity Cache / L2 residency);
//   * light item = one row of one slice: lane l owns the V-float vectors at
//     features (slice*C + c)*64V + l*V, c in [0, C): C*V accumulators/lane;
//     each nonzero's X row segment is read as 64V-float coalesced loads;
//   * heavy item = one 64-float sub-chunk of a row with > heavy_threshold
//     nonzeros: power-law hubs run on 2..C*V waves per slice with UH nonzeros
//     in flight each, scheduled first in their slice (sgc_plan_build sorts
//     them by degree), still one FMA chain per element;
//   * (col, val) of 64 consecutive nonzeros are read with one coalesced
//     256-B load each, then broadcast per nonzero with v_readlane into SGPRs,
//     so the X row base address is wave-uniform;
//   * U nonzeros are in flight per wave before their FMAs (U*C*V registers);
//     TLP (up to 8 waves/SIMD) hides the rest of the HBM/MALL latency.
//
// Work items beyond F (ragged last chunk) load a valid address (feature 0)
// and are never stored, so no exec-mask branches sit in the inner loop.
#include "common.h"

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace sgc {

constexpr int kBlock = 256;  // threads per light/heavy workgroup

// CSR (col, val) loads (streamed once per slice).
template <typename T>
__device__ __forceinline__ T ld_meta(const T *p) {
    return *p;
}

// Software-pipelined form of row_chunks: the X segments of step s+1 (U
// nonzeros) are issued before the FMAs of step s, so a wave always has one
// to two steps of gathers in flight instead of draining to zero between
// steps; the (col, val) block of the next 64 nonzeros is loaded one block
// ahead.  Loads are never predicated (a predicated load's phi copy would
// wait for every load in flight): indices past the row clamp to its last
// nonzero (same lines, no extra traffic) and only the FMAs are skipped, with
// wave-uniform branches.  Same FMA order as row_chunks.
template <int V, int C, int U>
__device__ __forceinline__ void row_chunks_pipe(const int *__restrict__ col,
                                                const float *__restrict__ val, int k0, int k1,
                                                const float *__restrict__ X, int64_t ldx,
                                                float *__restrict__ yrow, int F, int chunk0,
                                                int lane, bool accum) {
    using VT = typename Vec<V>::T;
    constexpr int kSteps = kWave / U;  // steps per 64-nonzero block
    static_assert(kWave % U == 0 && kSteps % 2 == 0, "U must divide 64 into an even count");
    if (accum && k1 == k0) return;  // nothing to add: the row keeps its partial chains
    uint32_t boff[C];
    bool ok[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int f = (chunk0 + c) * (kWave * V) + lane * V;
        ok[c] = f < F;
        boff[c] = ok[c] ? uint32_t(f) * 4u : 0u;
    }
    VT acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int v = 0; v < V; ++v) set_elem<V>(acc[c], v, 0.0f);
    if (accum) {  // continue the chains an earlier column-block pass stored
        const char *Yr = reinterpret_cast<const char *>(yrow);
#pragma unroll
        for (int c = 0; c < C; ++c)
            if (ok[c]) acc[c] = *reinterpret_cast<const VT *>(Yr + boff[c]);
    }

    if (k1 > k0) {
        const char *Xb = reinterpret_cast<const char *>(X);
        const int64_t row_bytes = ldx * 4;
        const int last = k1 - 1;
        // (col, val) of blocks b (A) and b+1 (B); clamped, never predicated
        int colA = ld_meta(col + min(k0 + lane, last));
        float valA = ld_meta(val + min(k0 + lane, last));
        int colB = ld_meta(col + min(k0 + kWave + lane, last));
        float valB = ld_meta(val + min(k0 + kWave + lane, last));
        VT xv[2][U][C];
        float vv[2][U];
        // step (block base, step i) -> buffer i & 1; lanes of the block in colA/colB
        auto issue = [&](int base, int i, int colr, float valr, int buf) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = min(base + i * U + u, last);
                const int l = (k - base) & (kWave - 1);  // clamped past the row: any lane
                                                         // of colr holds a valid column
                const int cj = __builtin_amdgcn_readlane(colr, l);
                vv[buf][u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(valr), l));
                const char *xr = Xb + (int64_t)cj * row_bytes;
#pragma unroll
                for (int c = 0; c < C; ++c)
                    xv[buf][u][c] = *reinterpret_cast<const VT *>(xr + boff[c]);
            }
        };
        issue(k0, 0, colA, valA, 0);
        for (int base = k0;; base += kWave) {
#pragma unroll
            for (int i = 0; i < kSteps; ++i) {
                const int cur = base + i * U;
                if (cur > last) break;  // uniform; the step issued for it is dropped
                if (i + 1 < kSteps)
                    issue(base, i + 1, colA, valA, (i + 1) & 1);
                else  // first step of the next block, from its prefetched (col, val)
                    issue(base + kWave, 0, colB, valB, 0);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (cur + u <= last) {
#pragma unroll
                        for (int c = 0; c < C; ++c)
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                set_elem<V>(acc[c], v,
                                            __builtin_fmaf(vv[i & 1][u],
                                                           lane_elem<V>(xv[i & 1][u][c], v),
                                                           lane_elem<V>(acc[c], v)));
                    }
                }
            }
            if (base + kWave > last) break;
            colA = colB;
            valA = valB;
            colB = ld_meta(col + min(base + 2 * kWave + lane, last));
            valB = ld_meta(val + min(base + 2 * kWave + lane, last));
        }
    }
    char *Yb = reinterpret_cast<char *>(yrow);
#pragma unroll
    for (int c = 0; c < C; ++c)
        if (ok[c]) *reinterpret_cast<VT *>(Yb + boff[c]) = acc[c];
}

// row_chunks_pipe scheduled like row_pairs_pipe: whole 64-nonzero blocks
// without an exit inside them (the compiler then keeps two steps of gathers
// in flight instead of draining to zero between steps), the last block stops
// at the row's end, the (col, val) block after next is loaded before the
// gathers of the step that starts the next block.  Same FMA order.
template <int V, int C, int U>
__device__ __forceinline__ void row_chunks_pipe2(const int *__restrict__ col,
                                                 const float *__restrict__ val, int k0, int k1,
                                                 const float *__restrict__ X, int64_t ldx,
                                                 float *__restrict__ yrow, int F, int chunk0,
                                                 int lane, bool accum) {
    using VT = typename Vec<V>::T;
    constexpr int kSteps = kWave / U;
    static_assert(kWave % U == 0 && kSteps % 2 == 0, "U must divide 64 into an even count");
    if (accum && k1 == k0) return;
    uint32_t boff[C];
    bool ok[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int f = (chunk0 + c) * (kWave * V) + lane * V;
        ok[c] = f < F;
        boff[c] = ok[c] ? uint32_t(f) * 4u : 0u;
    }
    VT acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int v = 0; v < V; ++v) set_elem<V>(acc[c], v, 0.0f);
    if (accum) {
        const char *Yr = reinterpret_cast<const char *>(yrow);
#pragma unroll
        for (int c = 0; c < C; ++c)
            if (ok[c]) acc[c] = *reinterpret_cast<const VT *>(Yr + boff[c]);
    }
    if (k1 > k0) {
        const char *Xb = reinterpret_cast<const char *>(X);
        const int64_t row_bytes = ldx * 4;
        const int last = k1 - 1;
        int colA = ld_meta(col + min(k0 + lane, last));
        float valA = ld_meta(val + min(k0 + lane, last));
        int colB = ld_meta(col + min(k0 + kWave + lane, last));
        float valB = ld_meta(val + min(k0 + kWave + lane, last));
        VT xv[2][U][C];
        float vv[2][U];
        auto issue = [&](int base, int i, int colr, float valr, int buf) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = min(base + i * U + u, last);
                const int l = (k - base) & (kWave - 1);
                const int cj = __builtin_amdgcn_readlane(colr, l);
                vv[buf][u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(valr), l));
                const char *xr = Xb + (int64_t)cj * row_bytes;
#pragma unroll
                for (int c = 0; c < C; ++c)
                    xv[buf][u][c] = *reinterpret_cast<const VT *>(xr + boff[c]);
            }
        };
        auto step = [&](int base, int i, bool last_block) {
            const int cur = base + i * U;
            if (i + 1 < kSteps) {
                issue(base, i + 1, colA, valA, (i + 1) & 1);
            } else if (!last_block) {
                const int nb2 = base + 2 * kWave;  // the block after next
                const int cN = ld_meta(col + min(nb2 + lane, last));
                const float vN = ld_meta(val + min(nb2 + lane, last));
                issue(base + kWave, 0, colB, valB, 0);
                colA = colB;
                valA = valB;
                colB = cN;
                valB = vN;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (cur + u <= last) {
#pragma unroll
                    for (int c = 0; c < C; ++c)
#pragma unroll
                        for (int v = 0; v < V; ++v)
                            set_elem<V>(acc[c], v,
                                        __builtin_fmaf(vv[i & 1][u],
                                                       lane_elem<V>(xv[i & 1][u][c], v),
                                                       lane_elem<V>(acc[c], v)));
                }
            }
        };
        issue(k0, 0, colA, valA, 0);
        const int nblk = (k1 - k0 + kWave - 1) / kWave;
        int base = k0;
        for (int b = 0; b + 1 < nblk; ++b, base += kWave) {
#pragma unroll
            for (int i = 0; i < kSteps; ++i) step(base, i, false);
        }
#pragma unroll
        for (int i = 0; i < kSteps; ++i)  // no exit: skipped steps fall through
            if (base + i * U <= last) step(base, i, true);
    }
    char *Yb = reinterpret_cast<char *>(yrow);
#pragma unroll
    for (int c = 0; c < C; ++c)
        if (ok[c]) *reinterpret_cast<VT *>(Yb + boff[c]) = acc[c];
}

// Heavy row of the multi-row kernel, two nonzeros per load instruction: lanes
// 0-31 gather nonzero k's X segment, lanes 32-63 nonzero k+1's (16-B lanes,
// up to 128 floats per half), so one global_load_dwordx4 moves up to 1 KB
// (a one-row-per-instruction wave moves at most half that, and only the row
// width -- 304 B at a 76-float feature block).  v_permlane32_swap then gives
// every lane both values of its features (lo = x_k, hi = x_k+1) and the chain
// takes them in order, acc = fma(v_k, x_k, acc); acc = fma(v_k+1, x_k+1, acc):
// the same sequential FMA chain per element as one nonzero at a time (both
// halves compute it; the low half stores).  U pairs per step, two steps in
// flight (2U nonzeros each); (col, val) of 64 consecutive nonzeros in one VGPR
// per lane, the next block loaded one ahead.  Indices past the row clamp to
// its last nonzero (never out of bounds) and their FMAs are skipped.
constexpr int kPairsU = 4;  // nonzero pairs per step (8 nonzeros; 16 in flight)

// Schedule: every 64-nonzero block but the last runs all its steps (no exit
// inside a block, so the compiler's wait counts keep two steps in flight
// instead of draining the loads at every block -- with per-step exits they
// did), the last block stops at the row's end; the (col, val) block after
// next is loaded before the gathers of the step that starts the next block.
// Reddit shape K=2: 9.01 -> 8.94 ms, bit-identical (profiles/r03/s5/pairs.log).
//
// TR (transposed pairs, heavy_pairs bit 16): one v_permlane32_swap per two
// registers instead -- (r0, r2) and (r1, r3) -- leaves lane (h, j) (h = lane
// >= 32) with features 4j+2h, 4j+2h+1 of both nonzeros, so each lane runs
// two chains (its two features) at one FMA per nonzero each: two swaps and
// four FMAs per pair where the untransposed form spends four and eight (both
// halves computing every chain); every lane stores its two features.
template <int U, bool O32, bool TR = false>
__device__ __forceinline__ void row_pairs_pipe(const int *__restrict__ col,
                                               const float *__restrict__ val, int k0, int k1,
                                               const float *__restrict__ X, int64_t ldx,
                                               float *__restrict__ yrow, int F, int f_lane,
                                               bool lane_ok, bool vec_store, int lane,
                                               bool accum) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int kPairs = kWave / (2 * U);  // steps per 64-nonzero block
    static_assert(kWave % (2 * U) == 0 && kPairs % 2 == 0, "2U must divide 64 into an even count");
    if (accum && k1 == k0) return;
    typedef float f2 __attribute__((ext_vector_type(2)));
    const bool hi = lane >= 32;
    const uint32_t boff = lane_ok ? uint32_t(f_lane) * 4u : 0u;
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    f2 acc2 = {0.0f, 0.0f};           // TR: features fo, fo + 1
    const int fo = f_lane + (hi ? 2 : 0);
    if (accum && lane_ok) {
        if constexpr (TR) {
            if (vec_store) {
                acc2 = *reinterpret_cast<const f2 *>(yrow + fo);
            } else {
#pragma unroll
                for (int v = 0; v < 2; ++v)
                    if (fo + v < F) acc2[v] = yrow[fo + v];
            }
        } else if (vec_store) {
            acc = *reinterpret_cast<const f4 *>(yrow + f_lane);
        } else {
#pragma unroll
            for (int v = 0; v < 4; ++v)
                if (f_lane + v < F) acc[v] = yrow[f_lane + v];
        }
    }
    if (k1 > k0) {
        const char *Xb = reinterpret_cast<const char *>(X);
        const int64_t row_bytes = ldx * 4;
        const int last = k1 - 1;
        int colA = ld_meta(col + min(k0 + lane, last));
        float valA = ld_meta(val + min(k0 + lane, last));
        int colB = ld_meta(col + min(k0 + kWave + lane, last));
        float valB = ld_meta(val + min(k0 + kWave + lane, last));
        f4 xv[2][U];
        float v0[2][U], v1[2][U];
        auto issue = [&](int base, int i, int colr, float valr, int buf) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int ka = min(base + i * 2 * U + 2 * u, last);
                const int kb = min(ka + 1, last);
                const int la = (ka - base) & (kWave - 1), lb = (kb - base) & (kWave - 1);
                const int ca = __builtin_amdgcn_readlane(colr, la);
                const int cb = __builtin_amdgcn_readlane(colr, lb);
                v0[buf][u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(valr), la));
                v1[buf][u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(valr), lb));
                const int cj = hi ? cb : ca;
                if constexpr (O32)
                    xv[buf][u] = *reinterpret_cast<const f4 *>(
                        Xb + (__umul24((uint32_t)cj, (uint32_t)row_bytes) + boff));
                else
                    xv[buf][u] = *reinterpret_cast<const f4 *>(Xb + (int64_t)cj * row_bytes + boff);
            }
        };
        auto step = [&](int base, int i, bool last_block) {
            const int cur = base + i * 2 * U;
            if (i + 1 < kPairs) {
                issue(base, i + 1, colA, valA, (i + 1) & 1);
            } else if (!last_block) {
                const int nb2 = base + 2 * kWave;  // the block after next
                const int cN = ld_meta(col + min(nb2 + lane, last));
                const float vN = ld_meta(val + min(nb2 + lane, last));
                issue(base + kWave, 0, colB, valB, 0);
                colA = colB;
                valA = valB;
                colB = cN;
                valB = vN;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int ka = cur + 2 * u;
                if (ka > last) break;  // uniform
                if constexpr (TR) {
                    const f4 x = xv[i & 1][u];
                    const auto s02 = __builtin_amdgcn_permlane32_swap(
                        __float_as_uint(x[0]), __float_as_uint(x[2]), false, false);
                    const auto s13 = __builtin_amdgcn_permlane32_swap(
                        __float_as_uint(x[1]), __float_as_uint(x[3]), false, false);
                    acc2[0] = __builtin_fmaf(v0[i & 1][u], __uint_as_float(s02[0]), acc2[0]);
                    acc2[1] = __builtin_fmaf(v0[i & 1][u], __uint_as_float(s13[0]), acc2[1]);
                    if (ka + 1 <= last) {
                        acc2[0] = __builtin_fmaf(v1[i & 1][u], __uint_as_float(s02[1]), acc2[0]);
                        acc2[1] = __builtin_fmaf(v1[i & 1][u], __uint_as_float(s13[1]), acc2[1]);
                    }
                    continue;
                }
                f4 xa, xb;
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const uint32_t x = __float_as_uint(xv[i & 1][u][v]);
                    const auto t = __builtin_amdgcn_permlane32_swap(x, x, false, false);
                    xa[v] = __uint_as_float(t[0]);
                    xb[v] = __uint_as_float(t[1]);
                }
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[v] = __builtin_fmaf(v0[i & 1][u], xa[v], acc[v]);
                if (ka + 1 <= last) {
#pragma unroll
                    for (int v = 0; v < 4; ++v)
                        acc[v] = __builtin_fmaf(v1[i & 1][u], xb[v], acc[v]);
                }
            }
        };
        issue(k0, 0, colA, valA, 0);
        const int nblk = (k1 - k0 + kWave - 1) / kWave;
        int base = k0;
        for (int b = 0; b + 1 < nblk; ++b, base += kWave) {
#pragma unroll
            for (int i = 0; i < kPairs; ++i) step(base, i, false);
        }
#pragma unroll
        for (int i = 0; i < kPairs; ++i)  // no exit: skipped steps fall through
            if (base + i * 2 * U <= last) step(base, i, true);
    }
    if constexpr (TR) {
        if (lane_ok) {
            if (vec_store) {
                *reinterpret_cast<f2 *>(yrow + fo) = acc2;
            } else {
#pragma unroll
                for (int v = 0; v < 2; ++v)
                    if (fo + v < F) yrow[fo + v] = acc2[v];
            }
        }
    } else if (!hi && lane_ok) {
        if (vec_store) {
            *reinterpret_cast<f4 *>(yrow + f_lane) = acc;
        } else {
#pragma unroll
            for (int v = 0; v < 4; ++v)
                if (f_lane + v < F) yrow[f_lane + v] = acc[v];
        }
    }
}

// Heavy row of a NARROW launch (at most 64 floats), four nonzeros per load
// instruction: lane group g = lane / 16 gathers nonzero k+g's X segment,
// 16 lanes x V floats (V = 4 / 2 / 1: segments of up to 64 / 32 / 16 floats),
// so one load moves four row segments where pairs move two (at 64 floats
// pairs leave half of each 32-lane half idle, at 32 or 12 floats three
// quarters or more).  What bounds a narrow pass is the load instructions (a
// wave instruction costs the texture unit about the same whether it carries
// two or four segments: scripts/micro/gather_rate.hip, 64 floats 0.42 ms at two
// segments per instruction vs 0.37 at four) and a long row's loads in flight
// (4 x U x 2 here: twice the pairs').  Every lane then needs the four
// nonzeros' values of its features, in order:
//   v_permlane32_swap(x, x) -> t0 = x of lane L mod 32 (group 0 or 1, same
//     16-lane position), t1 = x of lane 32 + L mod 32 (group 2 or 3);
//   v_permlane16_swap(t, t) -> t of lane L & ~16 and of lane L | 16:
//     groups 0, 1 from t0 and 2, 3 from t1 -- in every lane, the same order;
// and the chain takes them in nonzero order: acc = fma(v_k, x_k, acc), ...,
// fma(v_k+3, x_k+3, acc), the same sequential FMA chain per element (all four
// groups compute it; group 0 stores).  The S values and column ids come from
// the 64-nonzero (col, val) block by v_readlane (wave-uniform), the column of
// the lane's own group by two selects.
constexpr int kQuadsU = 4;  // quads per step (16 nonzeros; two steps = 32 in flight)

template <int V, int U, bool O32>
__device__ __forceinline__ void row_quads_pipe(const int *__restrict__ col,
                                               const float *__restrict__ val, int k0, int k1,
                                               const float *__restrict__ X, int64_t ldx,
                                               float *__restrict__ yrow, int F, int f_lane,
                                               bool lane_ok, bool vec_store, int lane,
                                               bool accum) {
    using VT = typename Vec<V>::T;
    constexpr int kSteps = kWave / (4 * U);  // steps per 64-nonzero block
    static_assert(kWave % (4 * U) == 0 && kSteps % 2 == 0, "4U must divide 64 into an even count");
    if (accum && k1 == k0) return;
    const int g = lane >> 4;
    const uint32_t boff = lane_ok ? uint32_t(f_lane) * 4u : 0u;
    VT acc;
#pragma unroll
    for (int v = 0; v < V; ++v) set_elem<V>(acc, v, 0.0f);
    if (accum && lane_ok) {
        if (vec_store) {
            acc = *reinterpret_cast<const VT *>(yrow + f_lane);
        } else {
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (f_lane + v < F) set_elem<V>(acc, v, yrow[f_lane + v]);
        }
    }
    if (k1 > k0) {
        const char *Xb = reinterpret_cast<const char *>(X);
        const int64_t row_bytes = ldx * 4;
        const int last = k1 - 1;
        int colA = ld_meta(col + min(k0 + lane, last));
        float valA = ld_meta(val + min(k0 + lane, last));
        int colB = ld_meta(col + min(k0 + kWave + lane, last));
        float valB = ld_meta(val + min(k0 + kWave + lane, last));
        VT xv[2][U];
        float vq[2][U][4];
        auto issue = [&](int base, int i, int colr, float valr, int buf) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kq = base + i * 4 * U + 4 * u;
                int c[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int l = (min(kq + j, last) - base) & (kWave - 1);
                    c[j] = __builtin_amdgcn_readlane(colr, l);
                    vq[buf][u][j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(valr), l));
                }
                const int c01 = (g & 1) ? c[1] : c[0];
                const int c23 = (g & 1) ? c[3] : c[2];
                const int cj = (g & 2) ? c23 : c01;
                if constexpr (O32)
                    xv[buf][u] = *reinterpret_cast<const VT *>(
                        Xb + (__umul24((uint32_t)cj, (uint32_t)row_bytes) + boff));
                else
                    xv[buf][u] = *reinterpret_cast<const VT *>(Xb + (int64_t)cj * row_bytes + boff);
            }
        };
        auto step = [&](int base, int i, bool last_block) {
            const int cur = base + i * 4 * U;
            if (i + 1 < kSteps) {
                issue(base, i + 1, colA, valA, (i + 1) & 1);
            } else if (!last_block) {
                const int nb2 = base + 2 * kWave;  // the block after next
                const int cN = ld_meta(col + min(nb2 + lane, last));
                const float vN = ld_meta(val + min(nb2 + lane, last));
                issue(base + kWave, 0, colB, valB, 0);
                colA = colB;
                valA = valB;
                colB = cN;
                valB = vN;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kq = cur + 4 * u;
                if (kq > last) break;  // uniform
                const int n_here = min(4, last - kq + 1);  // uniform
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const uint32_t x = __float_as_uint(lane_elem<V>(xv[i & 1][u], v));
                    const auto t = __builtin_amdgcn_permlane32_swap(x, x, false, false);
                    const auto p = __builtin_amdgcn_permlane16_swap(t[0], t[0], false, false);
                    const auto q = __builtin_amdgcn_permlane16_swap(t[1], t[1], false, false);
                    float a = lane_elem<V>(acc, v);
                    a = __builtin_fmaf(vq[i & 1][u][0], __uint_as_float(p[0]), a);
                    if (n_here > 1) a = __builtin_fmaf(vq[i & 1][u][1], __uint_as_float(p[1]), a);
                    if (n_here > 2) a = __builtin_fmaf(vq[i & 1][u][2], __uint_as_float(q[0]), a);
                    if (n_here > 3) a = __builtin_fmaf(vq[i & 1][u][3], __uint_as_float(q[1]), a);
                    set_elem<V>(acc, v, a);
                }
            }
        };
        issue(k0, 0, colA, valA, 0);
        const int nblk = (k1 - k0 + kWave - 1) / kWave;
        int base = k0;
        for (int b = 0; b + 1 < nblk; ++b, base += kWave) {
#pragma unroll
            for (int i = 0; i < kSteps; ++i) step(base, i, false);
        }
#pragma unroll
        for (int i = 0; i < kSteps; ++i)  // no exit: skipped steps fall through
            if (base + i * 4 * U <= last) step(base, i, true);
    }
    if (g == 0 && lane_ok) {
        if (vec_store) {
            *reinterpret_cast<VT *>(yrow + f_lane) = acc;
        } else {
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (f_lane + v < F) yrow[f_lane + v] = lane_elem<V>(acc, v);
        }
    }
}

// Heavy row of a 33..64-float launch, four nonzeros per load, TRANSPOSED: lane
// (g, j) (g = lane / 16, j = lane & 15) gathers floats 4j..4j+3 of nonzero
// k+g's segment -- one load moves four 256-B segments, as the light rows' do
// at this width -- and then a 4 x 4 transpose across the four lane groups
// (two v_permlane32_swap: g <-> g^2, two v_permlane16_swap: g <-> g^1) leaves
// lane (g, j) with feature 4j+g of the four nonzeros, in nonzero order:
//   after the 32-swaps (r0,r2), (r1,r3): g < 2 holds f0,f1 of nonzeros g, g+2;
//     g >= 2 holds f2,f3 of nonzeros g-2, g;
//   after the 16-swaps (r0,r1), (r2,r3): r0..r3 = feature 4j+g of nonzeros
//     k..k+3.
// Each lane then runs ONE chain (its feature) with one FMA per nonzero:
// four swaps + four FMAs per four nonzeros, where row_quads_pipe at V = 4
// spends twelve permutes and sixteen FMAs (every group recomputing every
// chain) -- the reason it lost to the pairs at 48-64 floats.  The chain is
// the same sequential fmaf chain per element; every lane stores its feature.
template <int U, bool O32>
__device__ __forceinline__ void row_quadsT_pipe(const int *__restrict__ col,
                                                const float *__restrict__ val, int k0, int k1,
                                                const float *__restrict__ X, int64_t ldx,
                                                float *__restrict__ yrow, int F, int f_lane,
                                                bool lane_ok, int lane, bool accum) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int kSteps = kWave / (4 * U);  // steps per 64-nonzero block
    static_assert(kWave % (4 * U) == 0 && kSteps % 2 == 0, "4U must divide 64 into an even count");
    if (accum && k1 == k0) return;
    const int g = lane >> 4;
    const int fo = f_lane + g;  // this lane's output feature
    const bool own = lane_ok && fo < F;
    const uint32_t boff = lane_ok ? uint32_t(f_lane) * 4u : 0u;
    float acc = 0.0f;
    if (accum && own) acc = yrow[fo];
    if (k1 > k0) {
        const char *Xb = reinterpret_cast<const char *>(X);
        const int64_t row_bytes = ldx * 4;
        const int last = k1 - 1;
        int colA = ld_meta(col + min(k0 + lane, last));
        float valA = ld_meta(val + min(k0 + lane, last));
        int colB = ld_meta(col + min(k0 + kWave + lane, last));
        float valB = ld_meta(val + min(k0 + kWave + lane, last));
        f4 xv[2][U];
        float vq[2][U][4];
        auto issue = [&](int base, int i, int colr, float valr, int buf) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kq = base + i * 4 * U + 4 * u;
                int c[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int l = (min(kq + j, last) - base) & (kWave - 1);
                    c[j] = __builtin_amdgcn_readlane(colr, l);
                    vq[buf][u][j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(valr), l));
                }
                const int c01 = (g & 1) ? c[1] : c[0];
                const int c23 = (g & 1) ? c[3] : c[2];
                const int cj = (g & 2) ? c23 : c01;
                if constexpr (O32)
                    xv[buf][u] = *reinterpret_cast<const f4 *>(
                        Xb + (__umul24((uint32_t)cj, (uint32_t)row_bytes) + boff));
                else
                    xv[buf][u] = *reinterpret_cast<const f4 *>(Xb + (int64_t)cj * row_bytes + boff);
            }
        };
        auto step = [&](int base, int i, bool last_block) {
            const int cur = base + i * 4 * U;
            if (i + 1 < kSteps) {
                issue(base, i + 1, colA, valA, (i + 1) & 1);
            } else if (!last_block) {
                const int nb2 = base + 2 * kWave;  // the block after next
                const int cN = ld_meta(col + min(nb2 + lane, last));
                const float vN = ld_meta(val + min(nb2 + lane, last));
                issue(base + kWave, 0, colB, valB, 0);
                colA = colB;
                valA = valB;
                colB = cN;
                valB = vN;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int kq = cur + 4 * u;
                if (kq > last) break;  // uniform
                const int n_here = min(4, last - kq + 1);  // uniform
                const f4 x = xv[i & 1][u];
                const auto s02 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x[0]),
                                                                  __float_as_uint(x[2]), false, false);
                const auto s13 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x[1]),
                                                                  __float_as_uint(x[3]), false, false);
                const auto t01 = __builtin_amdgcn_permlane16_swap(s02[0], s13[0], false, false);
                const auto t23 = __builtin_amdgcn_permlane16_swap(s02[1], s13[1], false, false);
                acc = __builtin_fmaf(vq[i & 1][u][0], __uint_as_float(t01[0]), acc);
                if (n_here > 1) acc = __builtin_fmaf(vq[i & 1][u][1], __uint_as_float(t01[1]), acc);
                if (n_here > 2) acc = __builtin_fmaf(vq[i & 1][u][2], __uint_as_float(t23[0]), acc);
                if (n_here > 3) acc = __builtin_fmaf(vq[i & 1][u][3], __uint_as_float(t23[1]), acc);
            }
        };
        issue(k0, 0, colA, valA, 0);
        const int nblk = (k1 - k0 + kWave - 1) / kWave;
        int base = k0;
        for (int b = 0; b + 1 < nblk; ++b, base += kWave) {
#pragma unroll
            for (int i = 0; i < kSteps; ++i) step(base, i, false);
        }
#pragma unroll
        for (int i = 0; i < kSteps; ++i)  // no exit: skipped steps fall through
            if (base + i * 4 * U <= last) step(base, i, true);
    }
    if (own) yrow[fo] = acc;
}

// Grid: x = work items of one feature slice, y = slice.  Workgroups are
// dispatched x-fastest, so the chip sweeps the slices one after another and
// only X[:, slice] (N x 64CV floats -- 119 MB at Reddit shape for 128
// floats) is live at a time: it stays in the 256 MB Infinity Cache and far
// more of it in the 4 MB per-XCD L2s than whole 2.4 KB rows would.  Within a
// slice the heavy rows come first (heaviest first), each split into
// 64-float sub-chunks (dword loads, UH nonzeros in flight) so a power-law hub
// is spread over 2C*V waves and finishes inside its slice.
#ifndef SGC_HEAVY_VEC
#define SGC_HEAVY_VEC 2
#endif
template <int HC, int NL, int IN>
__device__ __forceinline__ void hub_body(
    int bid, const int *__restrict__ row_ptr, const int *__restrict__ col,
    const float *__restrict__ val, const float *__restrict__ X, int64_t ldx,
    float *__restrict__ Y, int64_t ldy, int row_begin, int F, const int *__restrict__ hub_rows,
    int n_chunks, int accum);
constexpr int kFusedHubInstr = 8;  // (see HubShape)

// HF > 0: the serial hub rows fused into the launch (as spmm_rows_kernel's HF).
template <int V, int C, int U, int UH, int HF = 0>
__global__ __launch_bounds__(256) void spmm_csr_kernel(
    const int *__restrict__ row_ptr, const int *__restrict__ col, const float *__restrict__ val,
    const float *__restrict__ X, int64_t ldx, float *__restrict__ Y, int64_t ldy,
    int row_begin, int n_rows, int F, const int *__restrict__ heavy_rows, int n_heavy,
    int heavy_threshold, int accum, int heavy_pairs, const int *__restrict__ hub_rows = nullptr,
    int hub_chunks = 0, int n_hub_blocks = 0) {
    constexpr int VH = (SGC_HEAVY_VEC < V) ? SGC_HEAVY_VEC : V;  // heavy lanes' vector width
    constexpr int kSub = C * V / VH;  // 64*VH-float sub-chunks per slice (heavy items)
    int bx = (int)blockIdx.x;
    if constexpr (HF > 0) {
        if (bx < n_hub_blocks) {  // block-uniform
            if (blockIdx.y == 0)
                hub_body<HF, 3, kFusedHubInstr>(bx, row_ptr, col, val, X, ldx, Y, ldy, row_begin, F, hub_rows,
                                hub_chunks, accum);
            return;
        }
        bx -= n_hub_blocks;
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(
        (int)(bx * (blockDim.x / kWave) + (threadIdx.x / kWave)));
    const int slice = blockIdx.y;
    const int n_heavy_items = n_heavy * kSub;
    if (wave < n_heavy_items) {
        const int h = wave / kSub;
        const int sub = slice * kSub + (wave - h * kSub);  // in units of 64*VH floats
        if (sub * kWave * VH >= F) return;
        const int row = heavy_rows[h];
        const int k0 = row_ptr[row], k1 = row_ptr[row + 1];
        if constexpr (V == 4 && VH == 2) {
            if (heavy_pairs & 1) {  // the same 128-float sub-chunk, two nonzeros per load
                const int f = sub * 128 + (lane & 31) * 4;
                row_pairs_pipe<kPairsU, false>(col, val, k0, k1, X, ldx,
                                               Y + (int64_t)(row - row_begin) * ldy, F, f, f < F,
                                               true, lane, accum != 0);
                return;
            }
        }
        if (heavy_pairs & 2)
            row_chunks_pipe2<VH, 1, UH / VH>(col, val, k0, k1, X, ldx,
                                             Y + (int64_t)(row - row_begin) * ldy, F, sub, lane,
                                             accum != 0);
        else
            row_chunks_pipe<VH, 1, UH / VH>(col, val, k0, k1, X, ldx,
                                            Y + (int64_t)(row - row_begin) * ldy, F, sub, lane,
                                            accum != 0);
        return;
    }
    const int r = wave - n_heavy_items;
    if (r >= n_rows) return;
    const int row = row_begin + r;
    const int k0 = row_ptr[row], k1 = row_ptr[row + 1];
    if (k1 - k0 > heavy_threshold) return;  // done as a heavy item or by the hub kernel
    if (heavy_pairs & 2)
        row_chunks_pipe2<V, C, U>(col, val, k0, k1, X, ldx, Y + (int64_t)r * ldy, F, slice * C,
                                  lane, accum != 0);
    else
        row_chunks_pipe<V, C, U>(col, val, k0, k1, X, ldx, Y + (int64_t)r * ldy, F, slice * C,
                                 lane, accum != 0);
}

// ---------------------------------------------------------------------------
// Multi-row light kernel: LR lanes per row (8..32, a launch parameter), 4
// floats per lane (one global_load_dwordx4), R = 64 / LR rows per wavefront.
// A feature slice is LR * 4 floats: 128 at LR = 32 (2 rows per wave); a
// narrow launch -- a 76-float feature block, a 64-float group -- takes
// LR = width / 4 and a single slice, so up to 64 / LR rows share the wave
// instead of leaving most lanes idle.  (spmm_csr_kernel covers a 128-float
// slice with one row per wave and 8-B lanes: twice the load instructions for
// the same bytes, and at most one row per wave at any width.)
// It computes the columns up to F_load = F rounded up to 4: the engine's own
// 128-B-row buffers hold pad columns (don't-care values, computed like any
// other column, never returned); stores into a caller's buffer stop at F.
//  * each row's next LB (col, val) pairs are staged in a per-wave LDS block
//    (double buffered, loaded one block ahead); a lane reads U = 4 of its
//    row's ids and values with one ds_read_b128 each, a broadcast within the
//    row's LR lanes;
//  * U nonzeros per row per step, two steps in flight (software pipelined);
//  * the rows of one wave have different lengths: the wave runs to the
//    longest; lanes past their row's end re-load their row's last nonzero
//    (same lines, never out of bounds) and skip the FMAs -- still one
//    sequential FMA chain per element in CSR order.
// Heavy items (rows above heavy_threshold) come first in the grid, as in
// spmm_csr_kernel: one wave per 64*VH-float sub-chunk, n_sub per slice (8-B
// lanes at F % 4 != 0, one row per load instruction, twice the loads in
// flight per row; packing heavy rows R per wave like light rows measured 1.7x
// slower on a 76-float slice, profiles/r02/packed_sweep.log).
constexpr int kRowsU = 4;  // nonzeros per row per step (one b128 (col, val) read each)


// HF > 0: the fused rows + hub launch (small graphs whose hub chains are
// short, SGC_SPMM_HUB_SERIAL): the first n_hub_blocks workgroups of slice 0
// each run one (hub row, HF-float chunk) item of the hub kernel with three
// loader waves and the chain wave (hub_body<HF, 3>, the rows kernel's 256
// threads), every other workgroup the rows kernel's work -- one launch, so
// the hub chains run beside the light rows with no second launch and no
// cross-stream fork / join (Pubmed shape: the serial hub kernel added its
// whole 15 us chain to every hop).
template <int LB, int VH, int UH, bool O32, int QV, int HF = 0>
__global__ __launch_bounds__(256) void spmm_rows_kernel(
    const int *__restrict__ row_ptr, const int *__restrict__ col, const float *__restrict__ val,
    const float *__restrict__ X, int64_t ldx, float *__restrict__ Y, int64_t ldy,
    int row_begin, int n_rows, int F, int F_load, int LR, int vec_store, int n_sub,
    const int *__restrict__ heavy_rows, int n_heavy, int heavy_threshold, int accum,
    const int *__restrict__ light_rows, int heavy_pairs, const int *__restrict__ hub_rows = nullptr,
    int hub_chunks = 0, int n_hub_blocks = 0) {
    int bx = (int)blockIdx.x;
    if constexpr (HF > 0) {
        if (bx < n_hub_blocks) {  // block-uniform
            if (blockIdx.y == 0)
                hub_body<HF, 3, kFusedHubInstr>(bx, row_ptr, col, val, X, ldx, Y, ldy, row_begin, F, hub_rows,
                                hub_chunks, accum);
            return;
        }
        bx -= n_hub_blocks;
    }
    constexpr int V = 4, U = kRowsU < LB / 2 ? kRowsU : LB / 2;
    constexpr int kSteps = LB / U;  // steps per LDS block
    static_assert(kSteps >= 2 && kSteps % 2 == 0, "bad block");
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef int i4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) int s_col[kBlock / kWave][2][kWave];
    __shared__ __attribute__((aligned(16))) float s_val[kBlock / kWave][2][kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wl = threadIdx.x / kWave;
    const int wave = __builtin_amdgcn_readfirstlane((int)(bx * (kBlock / kWave) + wl));
    const int slice = blockIdx.y;
    const int R = kWave / LR;  // rows per wave (uniform)
    const int n_heavy_items = n_heavy * n_sub;
    if (wave < n_heavy_items) {
        const int h = wave / n_sub;
        const int row = heavy_rows[h];
        const int k0 = row_ptr[row], k1 = row_ptr[row + 1];
        if constexpr (QV == 4) {  // 16 lanes x 16 B per nonzero, transposed chains
            const int f = slice * (LR * V) + (lane & 15) * 4;
            row_quadsT_pipe<kQuadsU, O32>(col, val, k0, k1, X, ldx,
                                          Y + (int64_t)(row - row_begin) * ldy, F, f, f < F_load,
                                          lane, accum != 0);
            return;
        } else if constexpr (QV > 0) {  // 16 lanes per row: four nonzeros per load
            const int f = slice * (LR * V) + (lane & 15) * QV;
            row_quads_pipe<QV, kQuadsU, O32>(col, val, k0, k1, X, ldx,
                                             Y + (int64_t)(row - row_begin) * ldy, F, f,
                                             f < F_load, vec_store != 0, lane, accum != 0);
            return;
        }
        if (heavy_pairs & 1) {  // n_sub == 1: one item per (row, slice), two nonzeros per load
            const int j = lane & 31;
            const int f = slice * (LR * V) + j * V;
            if (heavy_pairs & 16)
                row_pairs_pipe<kPairsU, O32, true>(col, val, k0, k1, X, ldx,
                                                   Y + (int64_t)(row - row_begin) * ldy, F, f,
                                                   j < LR && f < F_load, vec_store != 0, lane,
                                                   accum != 0);
            else
                row_pairs_pipe<kPairsU, O32>(col, val, k0, k1, X, ldx,
                                             Y + (int64_t)(row - row_begin) * ldy, F, f,
                                             j < LR && f < F_load, vec_store != 0, lane, accum != 0);
            return;
        }
        const int sub = slice * n_sub + (wave - h * n_sub);  // in units of 64*VH floats
        if (sub * kWave * VH >= F) return;
        row_chunks_pipe<VH, 1, UH / VH>(col, val, k0, k1, X, ldx,
                                        Y + (int64_t)(row - row_begin) * ldy, F, sub, lane,
                                        accum != 0);
        return;
    }
    const int sub = lane / LR, l = lane - sub * LR;
    int r = 0, k0 = 0, len = 0;
    bool mine = false;
    if (light_rows) {  // light rows in the plan's order (n_rows of them here)
        const int w = wave - n_heavy_items;
        if (w * R >= n_rows) return;  // wave-uniform
        const int li = w * R + sub;
        if (sub < R && li < n_rows) {
            const int row = light_rows[li];
            r = row - row_begin;
            k0 = row_ptr[row];
            len = row_ptr[row + 1] - k0;
            mine = true;
        }
    } else {
        const int w = wave - n_heavy_items;
        if (w * R >= n_rows) return;  // wave-uniform
        r = w * R + sub;
        if (sub < R && r < n_rows) {
            k0 = row_ptr[row_begin + r];
            const int d = row_ptr[row_begin + r + 1] - k0;
            mine = d <= heavy_threshold;  // longer rows: heavy items / hub kernel
            len = mine ? d : 0;
        }
    }
    // the wave runs to its longest row; up to its shortest every step is
    // unpredicated (rows in length order make the two close)
    int n_max = 0, n_min = INT32_MAX;
    for (int s = 0; s < R; ++s) {
        const int ls = __builtin_amdgcn_readlane(len, s * LR);
        n_max = max(n_max, ls);
        n_min = min(n_min, ls);
    }
    const int f = slice * (LR * V) + l * V;
    const bool ok = sub < R && f < F_load;
    const uint32_t boff = ok ? uint32_t(f) * 4u : 0u;
    const int lds_row = (sub < R ? sub : 0) * LB;  // this lane's row block in LDS
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    // accumulate: continue the chains an earlier column-block pass stored;
    // rows without nonzeros in this pass are neither read nor written
    const bool store = mine && ok && (!accum || len > 0);
    if (accum && store) {
        const float *yr = Y + (int64_t)r * ldy;
        if (vec_store) {
            acc = *reinterpret_cast<const f4 *>(yr + f);
        } else {
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (f + v < F) acc[v] = yr[f + v];
        }
    }
    if (n_max > 0) {
        const char *Xb = reinterpret_cast<const char *>(X);
        const int64_t row_bytes = ldx * 4;
        // lanes l < LB stage (col, val) of their row's nonzero base + l,
        // clamped to its last one; a row without nonzeros reads X row 0 (its
        // FMAs are all skipped)
        const bool stager = sub < R && l < LB;
        // Never predicated: a conditional load makes (c, v) a phi whose
        // default copy must wait for every load in flight (s_waitcnt
        // vmcnt(0) once per block: the gathers of the steps ahead drained
        // at every LB nonzeros).  Lanes without a nonzero to stage read
        // nonzero 0 (valid: n_max > 0 means the CSR has one); the value is
        // either not staged or belongs to a row whose FMAs are all skipped.
        auto fetch = [&](int base, int &c, float &v) {
            const int kk = (len > 0 && l < LB) ? k0 + min(base + l, len - 1) : 0;
            c = col[kk];
            v = val[kk];
        };
        auto stage = [&](int buf, int c, float v) {
            if (stager) {
                s_col[wl][buf][lds_row + l] = c;
                s_val[wl][buf][lds_row + l] = v;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        int colB;
        float valB;
        {
            int c0;
            float v0;
            fetch(0, c0, v0);
            stage(0, c0, v0);
        }
        fetch(LB, colB, valB);
        f4 xv[2][U];
        float vv[2][U];
        auto issue = [&](int buf, int i, int slot) {
#pragma unroll
            for (int q = 0; q < U / 4; ++q) {
                const i4 cc =
                    *reinterpret_cast<const i4 *>(&s_col[wl][buf][lds_row + i * U + 4 * q]);
                const f4 vq =
                    *reinterpret_cast<const f4 *>(&s_val[wl][buf][lds_row + i * U + 4 * q]);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    vv[slot][4 * q + u] = vq[u];
                    if constexpr (O32)  // X spans < 4 GiB: 32-bit row offsets (saddr loads)
                        xv[slot][4 * q + u] = *reinterpret_cast<const f4 *>(
                            Xb + (__umul24((uint32_t)cc[u], (uint32_t)row_bytes) + boff));
                    else
                        xv[slot][4 * q + u] =
                            *reinterpret_cast<const f4 *>(Xb + (int64_t)cc[u] * row_bytes + boff);
                }
            }
        };
        issue(0, 0, 0);
        for (int base = 0;; base += LB) {
            const int buf = (base / LB) & 1;
#pragma unroll
            for (int i = 0; i < kSteps; ++i) {
                const int cur = base + i * U;
                if (cur >= n_max) break;  // wave-uniform
                if (i + 1 < kSteps) {
                    issue(buf, i + 1, (i + 1) & 1);
                } else {  // first step of the next block, from its prefetched (col, val)
                    stage(buf ^ 1, colB, valB);
                    issue(buf ^ 1, 0, 0);
                }
                if (cur + U <= n_min) {  // every row of the wave has these U (uniform)
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int v = 0; v < V; ++v)
                            acc[v] = __builtin_fmaf(vv[i & 1][u], xv[i & 1][u][v], acc[v]);
                } else {  // a row ends inside this step: per-lane predication
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (cur + u < len) {
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                acc[v] = __builtin_fmaf(vv[i & 1][u], xv[i & 1][u][v], acc[v]);
                        }
                    }
                }
            }
            if (base + LB >= n_max) break;
            fetch(base + 2 * LB, colB, valB);
        }
    }
    if (store) {
        float *yr = Y + (int64_t)r * ldy;
        if (vec_store) {
            *reinterpret_cast<f4 *>(yr + f) = acc;
        } else {
#pragma unroll
            for (int v = 0; v < V; ++v)
                if (f + v < F) yr[f + v] = acc[v];
        }
    }
}

// ---------------------------------------------------------------------------
// Hub rows (degree > hub_threshold): one 1024-thread workgroup per (row,
// HC-feature chunk).  A single wave's FMA chain over d nonzeros costs d FMAs
// -- cheap -- but a wave keeps only ~16 nonzeros' X segments in flight, so a
// 48k-nonzero hub on one wave runs ~3 ms, longer than a whole hop at P >= 2
// GPUs.  Here 15 loader waves gather X segments into an LDS double buffer
// while wave 0 runs the sequential chain out of LDS -- the same FMA order.
//
// The chain is the block's floor, so:
//  * wave 0 reads four nonzeros' X values per lane with one ds_read_b128 and
//    their four values with one broadcast ds_read_b128: the staging image is
//    transposed, gxT[feature][nonzero], row stride kStride = 4 mod 64 dwords
//    (conflict-free b128 reads per 16-lane group and b128 writes per 8-lane
//    group); each loader lane holds 16 CONSECUTIVE nonzeros of its feature
//    and writes them with four ds_write_b128;
//  * loaders keep kHubDepth rounds in registers: round t+kHubDepth is issued
//    while round t+1 is written, so a load has kHubDepth-1 rounds of FMA time
//    to land (a round is ~0.5 us of chain; an HBM/IC gather ~1-2 us), and the
//    column ids of a round arrive one round before its X loads.
// HC = 32 (one 128-B line per nonzero; lanes 32-63 load the second 16
// nonzeros of the loader's run) halves the bytes each block ingests per
// nonzero and spreads a hub over twice the CUs; it needs 128-B aligned X rows
// to stay one line per segment.
constexpr int kHubInstr = 16;  // consecutive nonzeros per loader lane per round
constexpr int kHubDepth = 3;   // rounds held in loader registers (17 loads each: vmcnt <= 63)
constexpr int kHubUnroll = 6;  // lcm(kHubDepth, 2): X ring slot and colv parity compile-time
constexpr int kHubPre = 4;     // LDS batches of 4 nonzeros the chain reads ahead

// The fused rows + hub launches (hub_body<HF, 3> inside spmm_csr_kernel /
// spmm_rows_kernel) stage IN = 8 nonzeros per loader lane: their LDS image is
// 18 KB instead of 35 KB, and since every workgroup of a launch carries it,
// eight workgroups (32 waves) fit a CU instead of four -- the light rows of a
// small graph are latency-bound and need the occupancy (Pubmed shape: the
// light rows alone ran 30.5 us per hop, fused at 35 KB 37.5 us).
template <int HC, int NL, int IN = kHubInstr>
struct HubShape {
    static_assert(IN % 4 == 0 && IN <= kHubInstr, "loader run: whole b128 LDS writes");
    static constexpr int kSegs = kWave / HC;                     // nonzero runs per loader wave
    static constexpr int kPerLoader = IN * kSegs;                // nonzeros per loader per round
    static constexpr int kRound = NL * kPerLoader;  // nonzeros per round (240 / 480 at NL = 15)
    static constexpr int kPad = 4 * kHubPre;        // read-ahead past kRound
    // dwords per gxT row: 4 mod 64 (conflict-free b128), and >= kRound + kPad
    // for the FMA loop's read-ahead (kHubPre batches of 4 past the last full batch)
    static constexpr int kStride = (kRound + kPad + 63) / 64 * 64 + 4;
};

#ifndef SGC_HUB_STAMPS
#define SGC_HUB_STAMPS 0  // diagnostic build only: per-round clock stamps of block 0
#endif
#if SGC_HUB_STAMPS
// [0] chain wave leaves the round's barrier, [1] chain wave reaches the next
// barrier (FMAs done), [2] loader wave 1 after its LDS store, [3] loader wave
// 1 reaches the barrier (loads issued); [4][0..1] s_memtime / s_memrealtime
// at kernel start and end (clock rate).  Lane 0's vector stores only; read
// back with sgc_debug_hub_stamps (exported by this build only).
constexpr int kStampRounds = 4096;
__device__ unsigned long long g_hub_stamp[5][kStampRounds];
#define HUB_STAMP(slot, r)                                                            \
    do {                                                                              \
        if (bid == 0 && lane == 0 && (r) < kStampRounds)                              \
            g_hub_stamp[slot][r] = __builtin_amdgcn_s_memtime();                      \
    } while (0)
#else
#define HUB_STAMP(slot, r) \
    do {                   \
    } while (0)
#endif

// The chain with the S values off the LDS-read path: one ds_read_b32 per 16
// nonzeros (lane l reads v[16i + (l & 15)], so each 16-lane row holds the
// iteration's 16 values) and every FMA takes its S value by a DPP row
// broadcast (v_fmac_f32_dpp ... row_newbcast:k): four LDS reads per 16
// nonzeros instead of eight.  Same operands and order as hub_chain_asm:
// acc = fma(v[k], x[k], acc).  X ring of four b128 slots (v80..v95) read four
// batches ahead; S in v96 (even iterations) / v97 (odd), read two iterations
// ahead (gv carries 32 floats of padding for it).  Invariant at the top of an
// iteration: outstanding LDS reads = [S_i, X0..X3, S_i+1].
__device__ __forceinline__ void hub_chain_dpp(float &acc, uint32_t xa, uint32_t vl, int iters,
                                              int rem) {
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n"
        "ds_read_b32 v96, %[vl]\n"
        "ds_read_b128 v[80:83], %[xa]\n"
        "ds_read_b128 v[84:87], %[xa] offset:16\n"
        "ds_read_b128 v[88:91], %[xa] offset:32\n"
        "ds_read_b128 v[92:95], %[xa] offset:48\n"
        "ds_read_b32 v97, %[vl] offset:64\n"
        "s_cmp_eq_u32 %[it], 0\n"
        "s_cbranch_scc1 2f\n"
        "1:\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v96, v80 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v81 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v82 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v83 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[80:83], %[xa] offset:64\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v96, v84 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v85 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v86 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v87 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[84:87], %[xa] offset:80\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v96, v88 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v89 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v90 row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v91 row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[88:91], %[xa] offset:96\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v96, v92 row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v93 row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v94 row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v95 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[92:95], %[xa] offset:112\n"
        "ds_read_b32 v96, %[vl] offset:128\n"
        "v_add_u32 %[xa], 64, %[xa]\n"
        "v_add_u32 %[vl], 64, %[vl]\n"
        "s_sub_u32 %[it], %[it], 1\n"
        "s_cmp_eq_u32 %[it], 0\n"
        "s_cbranch_scc1 3f\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v97, v80 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v81 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v82 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v83 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[80:83], %[xa] offset:64\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v97, v84 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v85 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v86 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v87 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[84:87], %[xa] offset:80\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v97, v88 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v89 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v90 row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v91 row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[88:91], %[xa] offset:96\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v97, v92 row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v93 row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v94 row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v95 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[92:95], %[xa] offset:112\n"
        "ds_read_b32 v97, %[vl] offset:128\n"
        "v_add_u32 %[xa], 64, %[xa]\n"
        "v_add_u32 %[vl], 64, %[vl]\n"
        "s_sub_u32 %[it], %[it], 1\n"
        "s_cmp_lg_u32 %[it], 0\n"
        "s_cbranch_scc1 1b\n"
        // even count done: the next iteration's S is in v96
        "2:\n"
        "s_cmp_gt_u32 %[rem], 0\n"
        "s_cbranch_scc0 5f\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v96, v80 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v81 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v82 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v83 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "s_cmp_gt_u32 %[rem], 1\n"
        "s_cbranch_scc0 5f\n"
        "s_waitcnt lgkmcnt(3)\n"
        "v_fmac_f32_dpp %[acc], v96, v84 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v85 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v86 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v87 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "s_cmp_gt_u32 %[rem], 2\n"
        "s_cbranch_scc0 5f\n"
        "s_waitcnt lgkmcnt(2)\n"
        "v_fmac_f32_dpp %[acc], v96, v88 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v89 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v90 row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v96, v91 row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "s_branch 5f\n"
        // odd count done: the next iteration's S is in v97
        "3:\n"
        "s_cmp_gt_u32 %[rem], 0\n"
        "s_cbranch_scc0 5f\n"
        "s_waitcnt lgkmcnt(4)\n"
        "v_fmac_f32_dpp %[acc], v97, v80 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v81 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v82 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v83 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "s_cmp_gt_u32 %[rem], 1\n"
        "s_cbranch_scc0 5f\n"
        "s_waitcnt lgkmcnt(3)\n"
        "v_fmac_f32_dpp %[acc], v97, v84 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v85 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v86 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v87 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "s_cmp_gt_u32 %[rem], 2\n"
        "s_cbranch_scc0 5f\n"
        "s_waitcnt lgkmcnt(2)\n"
        "v_fmac_f32_dpp %[acc], v97, v88 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v89 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v90 row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v97, v91 row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "s_branch 5f\n"
        "5:\n"
        "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [xa] "+v"(xa), [vl] "+v"(vl), [it] "+s"(iters)
        : [rem] "s"(rem)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91",
          "v92", "v93", "v94", "v95", "v96", "v97", "scc", "memory");
}

// NL loader waves + the chain wave per workgroup: 15 (1024 threads, ~133 KB
// of LDS: one workgroup per CU) or 7 (512 threads, ~68 KB: two per CU, half
// the CU held per hub chain; sgc_set_tuning("hub_loaders")).
// The body of one hub work item (hub row h, feature chunk c of block `bid`),
// shared by spmm_hub_kernel and the fused rows + hub launch of
// spmm_rows_kernel (HF > 0: NL = 3, the rows kernel's 256 threads).
template <int HC, int NL, int IN>
__device__ __forceinline__ void hub_body(
    int bid, const int *__restrict__ row_ptr, const int *__restrict__ col,
    const float *__restrict__ val, const float *__restrict__ X, int64_t ldx,
    float *__restrict__ Y, int64_t ldy, int row_begin, int F, const int *__restrict__ hub_rows,
    int n_chunks, int accum) {
    using Sh = HubShape<HC, NL, IN>;
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) float gxT[2][HC * Sh::kStride];  // 2 x 66.5 KB
    __shared__ __attribute__((aligned(16)))
    float gv[2][Sh::kRound + Sh::kPad + 32];  // + the DPP chain's S read-ahead
    const int lane = threadIdx.x & (kWave - 1);
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    // wave 0 runs the chain, waves 1..NL load (loader index li)
    const bool loader = w > 0;
    const int li = w - 1;
    const int h = bid / n_chunks;
    const int c = bid - h * n_chunks;
    const int row = hub_rows[h];
    const int k0 = row_ptr[row], k1 = row_ptr[row + 1];
    const int fl = lane & (HC - 1);  // feature within the chunk
    const int seg = lane / HC;       // which run of IN nonzeros (HC = 32: 0 or 1)
    const int f = c * HC + fl;
    const uint32_t boff = (f < F ? (uint32_t)f : 0u) * 4u;
    const char *Xb = reinterpret_cast<const char *>(X);
    const int64_t row_bytes = ldx * 4;
    const int n_round = (k1 - k0 + Sh::kRound - 1) / Sh::kRound;
    const int my_k = lane & (Sh::kPerLoader - 1);  // this lane's nonzero of the loader's run
    float regs[kHubDepth][IN];
    float vreg[kHubDepth];
    int colv[2];  // column ids of the loader's run, one per lane, for two future rounds
    // Loader waves only; `s` and `p` are compile-time constants after unrolling.
    // Column ids come in with ONE coalesced load per round (lane j holds
    // nonzero j's id, broadcast with v_readlane), issued a round before the X
    // loads that use them (per-nonzero scalar loads, each waited on, cost
    // ~0.4 us per round: 493 -> 406 us on the 47,857-nonzero row).
    auto load_col = [&](int r, int p) {
        const int kr = k0 + r * Sh::kRound + li * Sh::kPerLoader;
        colv[p] = col[min(kr + my_k, k1 - 1)];
    };
    auto load_x = [&](int r, int s, int p) {
        const int kr = k0 + r * Sh::kRound + li * Sh::kPerLoader;
#pragma unroll
        for (int j = 0; j < IN; ++j) {
            int cj = __builtin_amdgcn_readlane(colv[p], j);
            if (HC == 32) {
                const int c1 = __builtin_amdgcn_readlane(colv[p], IN + j);
                cj = seg ? c1 : cj;
            }
            regs[s][j] = *reinterpret_cast<const float *>(Xb + (int64_t)cj * row_bytes + boff);
        }
        vreg[s] = val[min(kr + my_k, k1 - 1)];
    };
    auto store = [&](int buf, int s) {
        f4 *dst = reinterpret_cast<f4 *>(
            &gxT[buf][fl * Sh::kStride + li * Sh::kPerLoader + seg * IN]);
#pragma unroll
        for (int q = 0; q < IN / 4; ++q)
            dst[q] = f4{regs[s][4 * q], regs[s][4 * q + 1], regs[s][4 * q + 2], regs[s][4 * q + 3]};
        if (lane < Sh::kPerLoader) gv[buf][li * Sh::kPerLoader + lane] = vreg[s];
    };
    // Loads are never predicated (rounds past the row re-read its last
    // nonzero): a conditional load makes its registers a phi, and copying a
    // phi waits for every load in flight.
    if (loader) {
#pragma unroll
        for (int s = 0; s < kHubDepth; ++s) {
            load_col(s, s & 1);
            load_x(s, s, s & 1);
        }
        load_col(kHubDepth, kHubDepth & 1);
        if (n_round > 0) store(0, 0);
    }
#if SGC_HUB_STAMPS
    if (bid == 0 && threadIdx.x == 0) {
        g_hub_stamp[4][0] = __builtin_amdgcn_s_memtime();
        g_hub_stamp[4][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    __syncthreads();
    float acc = 0.0f;
    if (accum && w == 0 && f < F) acc = Y[(int64_t)(row - row_begin) * ldy + f];
    for (int r0 = 0; r0 < n_round; r0 += kHubUnroll) {
#pragma unroll
        for (int s = 0; s < kHubUnroll; ++s) {
            // round t's X lives in regs[t % kHubDepth], its column ids in colv[t & 1]
            const int r = r0 + s;
            if (r >= n_round) break;  // block-uniform
            const int buf = r & 1;
            if (w == 0) HUB_STAMP(0, r);
            if (loader) {
                if (r + 1 < n_round) store(buf ^ 1, (s + 1) % kHubDepth);
                if (w == 1) HUB_STAMP(2, r);
                // ids of round r+D+1 first, so waiting for them (next round)
                // does not also wait for this round's X loads
                load_col(r + kHubDepth + 1, (s + kHubDepth + 1) & 1);
                load_x(r + kHubDepth, s % kHubDepth, (s + kHubDepth) & 1);
            } else if (w == 0) {
                const int n = min(Sh::kRound, k1 - (k0 + r * Sh::kRound));
                const int n4 = n >> 2;
                // LDS reads run kPre batches of four nonzeros ahead of the FMA
                // chain (a ds_read's ~64-cycle latency otherwise lands on the
                // chain every four FMAs); reads past n stay inside the padded
                // row / value buffers (kStride, gv) and are never used.
                // The chain as one asm loop (hub_chain_dpp): X values read
                // four batches of four nonzeros ahead with counted lgkmcnt
                // waits (left to the compiler the reads sink to one batch
                // ahead), the round's S values by one ds_read_b32 per 16
                // nonzeros and a DPP row broadcast per FMA.  Same FMA order.
                // What bounds it is one wave's LDS read rate: ~35 cycles per
                // 1-KB ds_read_b128 on gfx950 (scripts/micro/fma_chain.hip:
                // 9.5 cycles per nonzero alone, ~14-16 beside the loaders' LDS
                // writes; profiles/r02/micro_fma_chain_v2.log, hub_stamps.log).
                typedef __attribute__((address_space(3))) const float lds_f;
                const uint32_t xa = (uint32_t)(size_t)(lds_f *)(&gxT[buf][fl * Sh::kStride]);
                const uint32_t vl = (uint32_t)(size_t)(lds_f *)(&gv[buf][lane & 15]);
                hub_chain_dpp(acc, xa, vl, n4 >> 2, n4 & 3);
                const float *xt = &gxT[buf][fl * Sh::kStride];
                for (int kk = n4 * 4; kk < n; ++kk) acc = __builtin_fmaf(gv[buf][kk], xt[kk], acc);
            }
            if (w == 0) HUB_STAMP(1, r);
            if (w == 1) HUB_STAMP(3, r);
            __syncthreads();
        }
    }
    if (w == 0 && seg == 0 && f < F) Y[(int64_t)(row - row_begin) * ldy + f] = acc;
#if SGC_HUB_STAMPS
    if (bid == 0 && threadIdx.x == 0) {
        g_hub_stamp[4][2] = __builtin_amdgcn_s_memtime();
        g_hub_stamp[4][3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

template <int HC, int NL>
__global__ __launch_bounds__(64 * (NL + 1)) void spmm_hub_kernel(
    const int *__restrict__ row_ptr, const int *__restrict__ col, const float *__restrict__ val,
    const float *__restrict__ X, int64_t ldx, float *__restrict__ Y, int64_t ldy, int row_begin,
    int F, const int *__restrict__ hub_rows, int n_chunks, int accum) {
    hub_body<HC, NL, kHubInstr>((int)blockIdx.x, row_ptr, col, val, X, ldx, Y, ldy, row_begin, F,
                                hub_rows, n_chunks, accum);
}

namespace {

constexpr int kWavesPerBlock = kBlock / kWave;

struct LaunchArgs {
    const int *row_ptr;
    const int *col;
    const float *val;
    const float *X;
    int64_t ldx;
    float *Y;
    int64_t ldy;
    int row_begin, n_rows, F;
    const int *heavy_rows;
    int n_heavy, heavy_threshold;
    int slices;
    int accum;
    hipStream_t stream;
    const int *light_rows;  // SGC_SPMM_LIGHT_ORDER: the light rows in processing order, or null
    int n_light;
    // fused rows + hub launch (spmm_rows_kernel HF = 32): the hub rows and items
    const int *hub_rows = nullptr;
    int hub_chunks = 0, n_hub_blocks = 0;
};

// A side stream + fork/join events per (device, caller's stream) for the
// light kernel of a concurrent launch (the hub kernel stays on the caller's
// stream; the two are ordered against it by events, so the pair is
// capturable into a hipGraph).  One side stream per caller stream, so two
// callers' launches on different streams (the line partition's main and tail
// launches) never queue behind each other on a shared side stream.  The whole fork ->
// launch -> join sequence of one sgc_spmm call runs under `mu`: another host
// thread can neither re-record `fork` between this call's record and wait
// (which would order the hub kernel after the wrong stream) nor enqueue on
// the side stream while a capture holds it.
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    std::mutex mu;
};

// The side streams themselves come from a small per-device pool, created
// once (sgc_warmup creates it, with the loaders): hipStreamCreate took 7.8 ms
// for the process's first side stream (a new hardware queue), inside the first
// sgc_precompute the reference times (profiles/r06/s10: the first Reddit-shape
// call 16.2 ms against 8.2 on a second adjacency).  Caller streams take pool
// streams in turn; past kSidePool callers two callers share one (their light
// kernels then serialise on it: still correct, ordered by their own events).
constexpr int kSidePool = 4;
static std::mutex g_side_mu;

static hipError_t side_pool(int dev, hipStream_t **pool) {
    static std::map<int, std::vector<hipStream_t>> pools;
    std::vector<hipStream_t> &v = pools[dev];
    if (v.empty()) {
        // (a highest-priority side stream measured neutral, +-1%:
        // profiles/r01_hub_priority_sweep.log)
        for (int k = 0; k < kSidePool; ++k) {
            hipStream_t st = nullptr;
            hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
            if (e != hipSuccess) return e;
            v.push_back(st);
        }
    }
    *pool = v.data();
    return hipSuccess;
}

hipError_t warm_side_streams_impl() {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(g_side_mu);
    hipStream_t *pool = nullptr;
    return side_pool(dev, &pool);
}

hipError_t side_stream(SideStream **out, hipStream_t caller) {
    static std::map<std::pair<int, hipStream_t>, SideStream> per_dev;
    static std::map<int, int> next_pool;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(g_side_mu);
    SideStream &ss = per_dev[{dev, caller}];
    if (!ss.s) {
        hipStream_t *pool = nullptr;
        if ((e = side_pool(dev, &pool)) != hipSuccess) return e;
        if ((e = hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming)) != hipSuccess) return e;
        if ((e = hipEventCreateWithFlags(&ss.join, hipEventDisableTiming)) != hipSuccess) return e;
        ss.s = pool[next_pool[dev]++ % kSidePool];
    }
    *out = &ss;
    return hipSuccess;
}

// Launch timing (diagnostics, off by default; bench.py turns it on over its
// timed region): each launch_spmm records timing events around its
// light/heavy kernel and around its hub kernel, each on the stream the kernel
// runs on, so the two kernels' durations are measured separately.
// sgc_timing_collect() waits for and returns them.  Not for use inside a
// graph capture.
struct TimedLaunch {
    hipEvent_t l0 = nullptr, l1 = nullptr, h0 = nullptr, h1 = nullptr;
    int kernel = -1;  // light kernel: 0 spmm_csr_kernel, 1 spmm_rows_kernel, 2 / 3 the same with the hub rows fused, -1 none
    bool serial = false;  // hub kernel ran before the light kernel on the same stream
    bool hub_first = false;  // concurrent: hub kernel on the caller's stream, light on the side
};
static std::mutex g_timing_mu;
static bool g_timing = false;
static std::vector<TimedLaunch> g_timed;
static std::vector<hipEvent_t> g_event_pool;

// Launches recorded but not yet collected are capped: timing left on without
// sgc_timing_collect() stops recording instead of growing without bound.
constexpr size_t kMaxTimed = 1 << 16;

hipError_t pooled_event(hipEvent_t *e) {
    if (!g_event_pool.empty()) {
        *e = g_event_pool.back();
        g_event_pool.pop_back();
        return hipSuccess;
    }
    return hipEventCreate(e);
}

// Error-path guards of launch_spmm (called with g_timing_mu held while a
// TimedLaunch is filled): once the hub fork is recorded, the caller's stream
// is always joined to the side stream, and pooled timing events that never
// reached g_timed go back to the pool.
struct SideJoin {
    SideStream *side = nullptr;
    hipStream_t stream = nullptr;
    ~SideJoin() {
        if (!side) return;
        (void)hipEventRecord(side->join, side->s);
        (void)hipStreamWaitEvent(stream, side->join, 0);
    }
    hipError_t join() {  // the normal path: report the join's own errors
        SideStream *s = side;
        side = nullptr;
        hipError_t e = hipEventRecord(s->join, s->s);
        return e != hipSuccess ? e : hipStreamWaitEvent(stream, s->join, 0);
    }
};

struct TimedGuard {
    TimedLaunch *tl = nullptr;  // non-null while its events are not in g_timed
    ~TimedGuard() {
        if (!tl) return;
        for (hipEvent_t ev : {tl->l0, tl->l1, tl->h0, tl->h1})
            if (ev) g_event_pool.push_back(ev);
    }
    void commit() {
        g_timed.push_back(*tl);
        tl = nullptr;
    }
};

// Nonzeros per step: light items keep U*C*V <= ~40 registers of gathered X
// per step; heavy sub-chunk items go deeper (UH).  The pipelined loop holds
// two steps (measured best at 8 / 16: 48 VGPRs, 8 waves per SIMD, -3% per hop
// vs. an unpipelined U = 16 / 32; profiles/r01_sweep_pipe.log).
constexpr int kHeavyU = 16;

// Heavy rows, two nonzeros per load instruction (row_pairs_pipe, 16-B lanes)
// instead of one wave per 64*VH-float sub-chunk (row_chunks_pipe): bit 0 = in
// the multi-row kernel (Reddit shape K=2: 9.29 -> 9.12 ms, profiles/r03/s1/ab.log),
// bit 1 = in the one-row kernel; bit 2 = four nonzeros per load instead of two
// in the multi-row kernel on launches of <= 32 floats (row_quads_pipe); bit 3
// = the same on 33..64-float launches, transposed (row_quadsT_pipe: one
// 64-float hop over all Reddit-shape rows 0.715 -> 0.539 ms); bit 4 = the
// pairs transposed (row_pairs_pipe TR: 76 floats 0.775 -> 0.747 ms, 304
// floats 2.26 -> 2.16, Reddit K=2 8.11 -> 8.00; profiles/r04/quadsT_ab.log,
// pairsT_ab.log; all bit-identical).
// Set through sgc_set_tuning("heavy_pairs").
static int g_heavy_pairs = 29;
// One-row kernel: row_chunks_pipe2 (whole-block schedule) on launches of at
// least this many rows, row_chunks_pipe below.  Measured bit-identical,
// interleaved (profiles/r03/s5/chunks_*.log): RMAT shape K=3 (4.2 M rows)
// 95.5 -> 94.1 ms; Pubmed shape K=2 (19.7 k rows, latency-bound) 0.102 ->
// 0.109 ms.
constexpr int kChunksPipe2Rows = 1 << 20;

template <int V, int C, int HF = 0>
hipError_t launch_vc(const LaunchArgs &a) {
    constexpr int U0 = (C * V >= 16) ? 2 : (C * V >= 8) ? 4 : 8;
    constexpr int U = U0;
    constexpr int UH = kHeavyU;
    constexpr int VH = (SGC_HEAVY_VEC < V) ? SGC_HEAVY_VEC : V;
    const int64_t waves = (int64_t)a.n_heavy * (C * V / VH) + a.n_rows;
    const int64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock + (HF ? a.n_hub_blocks : 0);
    if (blocks >= INT32_MAX) return hipErrorInvalidValue;
    dim3 grid((unsigned)blocks, (unsigned)a.slices);
    hipLaunchKernelGGL((spmm_csr_kernel<V, C, U, UH, HF>), grid, dim3(kBlock), 0, a.stream,
                       a.row_ptr, a.col, a.val, a.X, a.ldx, a.Y, a.ldy, a.row_begin, a.n_rows,
                       a.F, a.heavy_rows, a.n_heavy, a.heavy_threshold, a.accum,
                       ((g_heavy_pairs >> 1) & 1) | (a.n_rows >= kChunksPipe2Rows ? 2 : 0),
                       a.hub_rows, a.hub_chunks, HF ? a.n_hub_blocks : 0);
    return hipGetLastError();
}

template <int V, int C>
hipError_t dispatch_c(int c, const LaunchArgs &a) {
    if constexpr (C == 0) {
        return hipErrorInvalidValue;
    } else {
        if (c == C) return launch_vc<V, C>(a);
        return dispatch_c<V, C - 1>(c, a);
    }
}

static int g_max_vec = 4;

// Light kernel choice when 16-B lanes are possible (F rounded up to 4 fits
// the rows and they are 16-B aligned): 0 = auto -- spmm_rows_kernel when
// spmm_csr_kernel could not use 16-B lanes itself (F % 4 != 0: Reddit's 602)
// or the launch is narrower than 128 floats or a large one at 128 / > 256
// floats (kWideRowsMin below), else spmm_csr_kernel (F = 152 .. 256, and
// Pubmed's 500: its one-row 256-float slices measured faster); 2 / 4 = always
// spmm_rows_kernel with 32 / 16 lanes per row on wide launches; 1 = never.
// profiles/r02/sweep_rows*.  Set through sgc_set_tuning("rows_per_wave").
static int g_rows_per_wave = 0;
// Large launches with 16-B lanes at F4 == 128 or F4 > 256 take the
// multi-row kernel (128-float slices, two rows per wave) even when
// spmm_csr_kernel could use 16-B lanes: one hop over the Reddit-shape graph
// (interleaved, bit-identical, profiles/r03/s10/ab_reddit.log) at 304 floats
// (the P = 2 feature block) 3.00 -> 2.50 ms, at 128 1.00 -> 0.94; at 152 / 160
// the one-row kernel's single 256-float slice stays faster (1.46 vs 1.60), and
// at 256 it is the RMAT shape's kernel (31.6 vs 37.3 ms per hop).  Small
// launches (Pubmed shape, F = 500) stay latency-bound on the one-row kernel.
constexpr int64_t kWideRowsMin = 65536;

template <int LB, int VH, bool O32, int QV, int HF = 0>
hipError_t launch_rows(const LaunchArgs &a, int F_load, int LR, int vec_store) {
    const int R = kWave / LR, SW = LR * 4;
    // each light row stages LB (col, val) pairs in its wave's 64-entry LDS block
    if (LR <= 0 || R * LB > kWave) return hipErrorInvalidValue;
    const int slices = (F_load + SW - 1) / SW;
    // heavy sub-chunks per slice (unpacked heavy rows): whole 64*VH-float
    // chunks of a slice, or of the launch's width when it is a single slice
    const int n_sub = (QV > 0 || (g_heavy_pairs & 1)) ? 1
                      : slices > 1 ? SW / (kWave * VH) : (F_load + kWave * VH - 1) / (kWave * VH);
    const int64_t heavy_waves = (int64_t)a.n_heavy * n_sub;
    // light items: every row (non-light rows skip themselves), or with a
    // light order exactly the light rows
    const int n_light_items = a.light_rows ? a.n_light : a.n_rows;
    const int64_t waves = heavy_waves + (n_light_items + R - 1) / R;
    const int64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock + (HF ? a.n_hub_blocks : 0);
    if (blocks >= INT32_MAX) return hipErrorInvalidValue;
    dim3 grid((unsigned)blocks, (unsigned)slices);
    hipLaunchKernelGGL((spmm_rows_kernel<LB, VH, kHeavyU, O32, QV, HF>), grid, dim3(kBlock), 0,
                       a.stream, a.row_ptr, a.col, a.val, a.X, a.ldx, a.Y, a.ldy, a.row_begin,
                       n_light_items, a.F, F_load, LR, vec_store, n_sub, a.heavy_rows, a.n_heavy,
                       a.heavy_threshold, a.accum, a.light_rows, g_heavy_pairs & 17, a.hub_rows,
                       a.hub_chunks, HF ? a.n_hub_blocks : 0);
    return hipGetLastError();
}

// Largest per-lane register vector the strides and base pointers allow.
int pick_vec(int64_t F, int64_t ldx, int64_t ldy, const void *X, const void *Y) {
    for (int V : {4, 2}) {
        if (V <= g_max_vec && F % V == 0 && ldx % V == 0 && ldy % V == 0 &&
            reinterpret_cast<uintptr_t>(X) % (4 * V) == 0 &&
            reinterpret_cast<uintptr_t>(Y) % (4 * V) == 0)
            return V;
    }
    return 1;
}

constexpr int max_chunks(int V) { return 16 / V; }  // <= 16 accumulators per lane

}  // namespace

// Feature-slice width in floats (rounded down to whole 64V-float chunks,
// at least one).  Default 128: one chunk per slice, so the chip's pass over
// S touches only X[:, slice] -- 119 MB at the Reddit shape, resident in the
// 256 MB MALL -- at the price of re-reading the CSR once per slice (8 B/nnz).
// Measured 4.74 ms/hop at the Reddit shape vs 5.48 ms for 256 and 6.24 ms
// for 0 = one slice as wide as the registers allow (2.9 GB live X)
// (profiles/r01_sweep_slices.log).  Set through sgc_set_tuning("slice_floats", n).
static int g_slice_floats = 128;
// Hub-kernel feature chunk: 0 = auto (32 on 128-B aligned X rows, else 64).
static int g_hub_chunk = 0;
// Where the hub kernel runs: 1 = concurrent with the light kernel -- the hub
// kernel on the caller's stream, the light kernel on a side stream (fork +
// join events: ~20-30 us of cross-queue synchronisation per launch); 2 = the
// caller's stream, before the light kernel (serial: costs the hub kernel's
// own time); 0 = per launch, serial when the caller sets SGC_SPMM_HUB_SERIAL
// (the Python layer does when the longest hub chain is shorter than that
// synchronisation: Pubmed shape 70 -> 61 us per hop), else concurrent.
// Concurrent launches put the HUB kernel on the caller's stream because the
// stream that waits on the fork event starts a few microseconds later: with
// the light kernel first, its 256-thread workgroups fill every CU and the
// 1024-thread hub workgroups trickled in as whole CUs drained, ending up to
// 0.26 ms after it (profiles/r03/s6 trace); hub first: Reddit K=2 8.96 ->
// 8.91 ms, one 76-float pass 0.91 -> 0.77 ms (profiles/r03/s7/stream3*.log).
// Set through sgc_set_tuning("hub_stream").
static int g_hub_stream = 0;
// Loader waves per hub workgroup: 15 or 7 (spmm_hub_kernel).  Set through
// sgc_set_tuning("hub_loaders").
static int g_hub_loaders = 15;
// Serial hub rows (SGC_SPMM_HUB_SERIAL) inside the multi-row kernel's launch
// (spmm_rows_kernel / spmm_csr_kernel HF = 32) instead of a hub kernel launch
// before it: 1 = on where the launch takes the multi-row kernel over whole
// 16-B-lane slices or the one-chunk csr kernel.  Set through
// sgc_set_tuning("hub_fuse").
static int g_hub_fuse = 1;

int set_tuning(const char *key, int64_t value) {
    SGC_REQUIRE(key, SGC_EINVAL, "set_tuning: null key");
    if (std::string(key) == "slice_floats") {
        SGC_REQUIRE(value >= 0 && value < (1 << 20), SGC_EINVAL, "slice_floats out of range");
        g_slice_floats = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "hub_chunk") {
        SGC_REQUIRE(value == 0 || value == 32 || value == 64, SGC_EINVAL,
                    "hub_chunk must be 0 (auto), 32 or 64");
        g_hub_chunk = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "hub_loaders") {
        SGC_REQUIRE(value == 7 || value == 15, SGC_EINVAL, "hub_loaders must be 7 or 15");
        g_hub_loaders = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "hub_fuse") {
        SGC_REQUIRE(value == 0 || value == 1, SGC_EINVAL, "hub_fuse must be 0 or 1");
        g_hub_fuse = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "hub_stream") {
        SGC_REQUIRE(value >= 0 && value <= 2, SGC_EINVAL, "hub_stream must be 0, 1 or 2");
        g_hub_stream = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "rows_per_wave") {
        SGC_REQUIRE(value == 0 || value == 1 || value == 2 || value == 4, SGC_EINVAL,
                    "rows_per_wave must be 0 (auto), 1, 2 or 4");
        g_rows_per_wave = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "heavy_pairs") {
        SGC_REQUIRE(value >= 0 && value <= 31, SGC_EINVAL, "heavy_pairs must be 0..31 (a bit mask)");
        g_heavy_pairs = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "tile_buffers") {
        SGC_REQUIRE(value == 1 || value == 2, SGC_EINVAL, "tile_buffers must be 1 or 2");
        g_tile_buffers = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "linear_ck") {
        SGC_REQUIRE(value == 32 || value == 64, SGC_EINVAL, "linear_ck must be 32 or 64");
        g_linear_ck = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "linear_kernel") {
        SGC_REQUIRE(value >= 0 && value <= 8, SGC_EINVAL, "linear_kernel must be 0..8");
        g_linear_kernel = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "backward_kernel") {
        SGC_REQUIRE(value >= 0 && value <= 3, SGC_EINVAL, "backward_kernel must be 0..3");
        g_backward_kernel = (int)value;
        return SGC_OK;
    }
    if (std::string(key) == "max_vec") {
        SGC_REQUIRE(value == 1 || value == 2 || value == 4, SGC_EINVAL, "max_vec must be 1, 2 or 4");
        g_max_vec = (int)value;
        return SGC_OK;
    }
    set_error("set_tuning: unknown key '%s'", key);
    return SGC_EINVAL;
}

int64_t get_tuning(const char *key) {
    if (key && std::string(key) == "slice_floats") return g_slice_floats;
    if (key && std::string(key) == "max_vec") return g_max_vec;
    if (key && std::string(key) == "heavy_pairs") return g_heavy_pairs;
    if (key && std::string(key) == "rows_per_wave") return g_rows_per_wave;
    if (key && std::string(key) == "hub_chunk") return g_hub_chunk;
    if (key && std::string(key) == "hub_stream") return g_hub_stream;
    if (key && std::string(key) == "hub_loaders") return g_hub_loaders;
    if (key && std::string(key) == "hub_fuse") return g_hub_fuse;
    if (key && std::string(key) == "tile_buffers") return g_tile_buffers;
    if (key && std::string(key) == "linear_kernel") return g_linear_kernel;
    if (key && std::string(key) == "linear_ck") return g_linear_ck;
    if (key && std::string(key) == "backward_kernel") return g_backward_kernel;
    return -1;
}

int launch_spmm(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                int64_t row_begin, int64_t row_end, const float *X, int64_t ldx, float *Y,
                int64_t ldy, int64_t F, const int32_t *heavy_rows, int64_t n_heavy,
                int64_t n_hub, int32_t heavy_threshold, uint32_t flags, hipStream_t stream) {
    // col_idx / val may be NULL for a CSR without nonzeros (torch's empty
    // tensors have no storage): the kernels never dereference them then
    SGC_REQUIRE(row_ptr && X && Y, SGC_EINVAL, "spmm: null pointer");
    SGC_REQUIRE(row_begin >= 0 && row_end >= row_begin && row_end < INT32_MAX, SGC_ERANGE,
                "spmm: bad row range [%lld, %lld)", (long long)row_begin, (long long)row_end);
    SGC_REQUIRE(F > 0 && F < (1 << 24), SGC_EINVAL, "spmm: bad feature count %lld", (long long)F);
    SGC_REQUIRE(ldx >= F && ldy >= F, SGC_EINVAL, "spmm: ldx/ldy (%lld/%lld) < F (%lld)",
                (long long)ldx, (long long)ldy, (long long)F);
    SGC_REQUIRE(n_heavy >= 0 && (n_heavy == 0 || heavy_rows), SGC_EINVAL, "spmm: bad plan");
    const int64_t n_rows = row_end - row_begin;
    if (n_rows == 0) return SGC_OK;
    // SGC_SPMM_LIGHT_ORDER: plan = [n_heavy heavy rows | the other rows in
    // processing order] (taken before the hub split below moves heavy_rows)
    const int *light_rows = nullptr;
    int64_t n_light = 0;
    if ((flags & SGC_SPMM_LIGHT_ORDER) && heavy_rows) {
        SGC_REQUIRE(n_heavy <= n_rows, SGC_EINVAL, "spmm: light order with n_heavy > rows");
        light_rows = heavy_rows + n_heavy;
        n_light = n_rows - n_heavy;
    }
    if (!heavy_rows) {
        n_heavy = 0;
        heavy_threshold = INT32_MAX;  // no plan: every row is a light item
    }
    n_hub = std::max<int64_t>(0, std::min<int64_t>(n_hub, n_heavy));
    if (flags & SGC_SPMM_NO_HUB) {  // hub rows are launched separately (SGC_SPMM_HUB_ONLY)
        heavy_rows += n_hub;
        n_heavy -= n_hub;
        n_hub = 0;
    }
    const bool hub_only = (flags & SGC_SPMM_HUB_ONLY) != 0;
    if (hub_only && n_hub == 0) return SGC_OK;
    const int accum = (flags & SGC_SPMM_ACCUMULATE) ? 1 : 0;
    SideStream *side = nullptr;
    std::unique_lock<std::mutex> side_lock;
    std::unique_lock<std::mutex> timing_lock(g_timing_mu);
    TimedLaunch tl;
    const bool timing = g_timing && g_timed.size() < kMaxTimed;
    if (!timing) timing_lock.unlock();
    // declared after the locks: destroyed (join, events back to the pool)
    // while they are still held
    TimedGuard timed_guard;
    if (timing) timed_guard.tl = &tl;
    SideJoin side_join;
    hipStream_t light_stream = stream;
    // hub kernel launch (on the caller's stream) of the n_hub rows at hub_rows
    const bool lines = ldx % 32 == 0 && reinterpret_cast<uintptr_t>(X) % 128 == 0;
    const int32_t *hub_rows = heavy_rows;
    auto launch_hub = [&](hipStream_t hs, int hc) -> hipError_t {
        const int n_chunks = (int)((F + hc - 1) / hc);
        const dim3 hub_grid((unsigned)(n_hub * n_chunks));
#define SGC_LAUNCH_HUB(HCV, NLV)                                                             \
    hipLaunchKernelGGL((spmm_hub_kernel<HCV, NLV>), hub_grid, dim3(64 * (NLV + 1)), 0, hs,   \
                       row_ptr, col_idx, val, X, ldx, Y, ldy, (int)row_begin, (int)F,        \
                       hub_rows, n_chunks, accum)
        if (hc == 32) {
            if (g_hub_loaders == 7) SGC_LAUNCH_HUB(32, 7);
            else SGC_LAUNCH_HUB(32, 15);
        } else {
            if (g_hub_loaders == 7) SGC_LAUNCH_HUB(64, 7);
            else SGC_LAUNCH_HUB(64, 15);
        }
#undef SGC_LAUNCH_HUB
        return hipGetLastError();
    };
    // 32-feature chunks spread a hub over more CUs; measured faster up to
    // F = 160 and slower from F = 320 (scripts/sweep_narrow.py), and they
    // need 128-B aligned rows to stay one line per segment.
    const int hub_hc = g_hub_chunk ? g_hub_chunk : (lines && F <= 192 ? 32 : 64);
    bool hub_deferred = false;  // serial hub rows left for the fused launch (or just before the light kernel)
    if (n_hub > 0) {
        // hub rows (the heaviest n_hub of the plan) run beside the light
        // kernel (g_hub_stream)
        SGC_REQUIRE(n_hub * ((F + 31) / 32) < (int64_t)INT32_MAX, SGC_ERANGE,
                    "spmm: too many hub items");
        const hipStream_t hs = stream;  // always the caller's stream
        const bool serial =
            g_hub_stream == 2 || (g_hub_stream == 0 && (flags & SGC_SPMM_HUB_SERIAL));
        // (the fused items read floats one at a time: any row alignment)
        hub_deferred = serial && !hub_only && g_hub_fuse && g_hub_chunk == 0;
        if (!hub_deferred) {
            if (!hub_only && !serial) {
                SGC_HIP_CHECK(side_stream(&side, stream));
                side_lock = std::unique_lock<std::mutex>(side->mu);
                SGC_HIP_CHECK(hipEventRecord(side->fork, stream));
                SGC_HIP_CHECK(hipStreamWaitEvent(side->s, side->fork, 0));
                side_join.side = side;  // from here on every exit joins
                side_join.stream = stream;
                light_stream = side->s;  // the hub kernel stays on the caller's stream
                tl.hub_first = true;
            }
            if (timing) {
                SGC_HIP_CHECK(pooled_event(&tl.h0));
                SGC_HIP_CHECK(pooled_event(&tl.h1));
                SGC_HIP_CHECK(hipEventRecord(tl.h0, hs));
                tl.serial = hs == light_stream;
            }
            SGC_HIP_CHECK(launch_hub(hs, hub_hc));
            if (timing) SGC_HIP_CHECK(hipEventRecord(tl.h1, hs));
        }
        heavy_rows += n_hub;
        n_heavy -= n_hub;
        if (hub_only) {
            if (timing) {  // no light kernel: an empty light interval
                SGC_HIP_CHECK(pooled_event(&tl.l0));
                SGC_HIP_CHECK(pooled_event(&tl.l1));
                SGC_HIP_CHECK(hipEventRecord(tl.l0, hs));
                SGC_HIP_CHECK(hipEventRecord(tl.l1, hs));
                timed_guard.commit();
            }
            return SGC_OK;
        }
    }
    // a deferred hub launch that the fused kernel does not take runs here,
    // serially before the light kernel, as it would have
    auto hub_before_light = [&]() -> int {
        if (timing) {
            SGC_HIP_CHECK(pooled_event(&tl.h0));
            SGC_HIP_CHECK(pooled_event(&tl.h1));
            SGC_HIP_CHECK(hipEventRecord(tl.h0, stream));
            tl.serial = true;
        }
        SGC_HIP_CHECK(launch_hub(stream, hub_hc));
        if (timing) SGC_HIP_CHECK(hipEventRecord(tl.h1, stream));
        return SGC_OK;
    };

    LaunchArgs a{row_ptr, col_idx, val, X, ldx, Y, ldy, (int)row_begin, (int)n_rows, (int)F,
                 heavy_rows, (int)n_heavy, heavy_threshold, 0, accum, light_stream};
    a.light_rows = light_rows;  // used by the multi-row kernel (the one-row kernel: natural order)
    a.n_light = (int)n_light;
    // 16-B lanes over F rounded up to 4 columns: X rows must be 16-B aligned
    // and readable that far (flag SGC_SPMM_X_PADDED unless F % 4 == 0)
    const int64_t F4 = (F + 3) / 4 * 4;
    const uintptr_t xa = reinterpret_cast<uintptr_t>(X), ya = reinterpret_cast<uintptr_t>(Y);
    const bool v4_ok = ldx % 4 == 0 && xa % 16 == 0 && F4 <= ldx && F4 >= 32 &&
                       (F4 == F || (flags & SGC_SPMM_X_PADDED));
    // With both buffers padded, the one-row kernel may compute F rounded up
    // to 4 as well: one 256-float slice (16-B lanes) covers a 129..256-float
    // launch that the multi-row kernel would run as two passes (128 + the
    // rest) -- e.g. a 146-column feature block at P = 4.  Wider launches keep
    // the multi-row kernel's 128-float slices (Reddit's 602: MALL residency).
    const bool pad_both = (flags & SGC_SPMM_X_PADDED) && (flags & SGC_SPMM_Y_PADDED);
    const int64_t F_csr =
        (F % 4 != 0 && pad_both && F4 > 128 && F4 <= 256 && F4 <= ldx && F4 <= ldy) ? F4 : F;
    const bool csr_v4 = F_csr % 4 == 0 && pick_vec(F_csr, ldx, ldy, X, Y) == 4;
    // Small, wide launches (Cora shape: 2,708 rows x 1,433 features, X in
    // L2): latency-bound, so fewer and wider work items win -- the one-row
    // kernel with 512-float slices, 19.7 vs 24.9 us per hop for the
    // 128-float rows kernel (profiles/r02/small_shapes_sweep.log).  Only at
    // the default schedule knobs.
    const bool small_wide = n_rows * F <= (int64_t(1) << 23) && F > 256 &&
                            g_rows_per_wave == 0 && g_slice_floats == 128;
    const bool wide_rows = n_rows >= kWideRowsMin && (F4 == 128 || F4 > 256);
    const bool rows_kernel = v4_ok && g_rows_per_wave != 1 && !small_wide &&
                             (g_rows_per_wave > 1 || !csr_v4 || F4 < 128 || wide_rows);
    hipError_t e = hipSuccess;
    if (rows_kernel) {
        const int vec_store = ldy % 4 == 0 && ya % 16 == 0 && F4 <= ldy &&
                              (F4 == F || (flags & SGC_SPMM_Y_PADDED));
        // lanes per row: the launch's width in 4-float lanes when it fits a
        // wave's half or less (one slice), else 32 (or 16 when forced)
        int LR = F4 >= 128 ? (g_rows_per_wave == 4 ? 16 : 32) : (int)(F4 / 4);
        if (LR > 32) LR = 32;
        const int SW = LR * 4;
        const bool multi = F4 > SW;
        const bool vh2 = F % 2 == 0 && ldx % 2 == 0 && ldy % 2 == 0 && xa % 8 == 0 &&
                         ya % 8 == 0 && (!multi || SW % (kWave * 2) == 0);
        SGC_REQUIRE(n_heavy * 8 + n_rows < (int64_t)INT32_MAX, SGC_ERANGE,
                    "spmm: too many work items");
        // the fused hub items need the 256-thread multi-row kernel with
        // 16-B lanes over whole slices (LR >= 16, two-float heavy sub-chunks)
        const bool fused = hub_deferred && LR >= 16 && vh2 && F4 > 64;
        if (hub_deferred && !fused) {
            const int rc = hub_before_light();
            if (rc != SGC_OK) return rc;
        }
        if (fused) {
            a.hub_rows = hub_rows;
            a.hub_chunks = (int)((F + 31) / 32);
            a.n_hub_blocks = (int)(n_hub * a.hub_chunks);
        }
        if (timing) {
            SGC_HIP_CHECK(pooled_event(&tl.l0));
            SGC_HIP_CHECK(pooled_event(&tl.l1));
            SGC_HIP_CHECK(hipEventRecord(tl.l0, light_stream));
            tl.kernel = fused ? 2 : 1;
        }
        // 32-bit row offsets (one full-rate 24-bit multiply per gathered row)
        // when the caller vouches that X spans < 4 GiB and has < 2^24 rows
        const bool o32 = (flags & SGC_SPMM_X_UNDER_4G) && ldx * 4 < (int64_t(1) << 24);
#define SGC_ROWS(LBV, VHV, QVV)                                                     \
    (o32 ? launch_rows<LBV, VHV, true, QVV>(a, (int)F4, LR, vec_store)              \
         : launch_rows<LBV, VHV, false, QVV>(a, (int)F4, LR, vec_store))
        // heavy rows four nonzeros per load (row_quads_pipe) on launches of at
        // most 32 floats; measured (one hop over all Reddit-shape rows,
        // interleaved, bit-identical, profiles/r04/quads_ab.log) 32 floats
        // 0.667 -> 0.615 ms, but 48 and 64 floats slower (0.68 -> 0.82, 0.72
        // -> 0.85) and 64-float slices at full width far slower (3.8 -> 5.8):
        // there the pairs stay
        int qv = ((g_heavy_pairs & 4) && LR <= 16 && F4 <= 32) ? (F4 > 16 ? 2 : 1) : 0;
        // 33..64 floats: the transposed quads (row_quadsT_pipe, heavy_pairs bit 8)
        if ((g_heavy_pairs & 8) && LR <= 16 && F4 > 32 && F4 <= 64) qv = 4;
        if (qv == 4)  // the light rows' LDS block: LB * rows per wave <= 64
            e = LR >= 16 ? SGC_ROWS(16, 2, 4) : SGC_ROWS(8, 2, 4);
        else if (qv == 2)
            e = SGC_ROWS(8, 2, 2);
        else if (qv == 1)
            e = SGC_ROWS(8, 2, 1);
        else if (fused)
            e = o32 ? launch_rows<16, 2, true, 0, 32>(a, (int)F4, LR, vec_store)
                    : launch_rows<16, 2, false, 0, 32>(a, (int)F4, LR, vec_store);
        else if (LR >= 16)
            e = vh2 ? SGC_ROWS(16, 2, 0) : SGC_ROWS(16, 1, 0);
        else
            e = vh2 ? SGC_ROWS(8, 2, 0) : SGC_ROWS(8, 1, 0);
#undef SGC_ROWS
    } else {
        const int V = pick_vec(F_csr, ldx, ldy, X, Y);
        a.F = (int)(V == 4 ? F_csr : F);  // pad columns only with 16-B lanes
        const int chunks_total = (int)((a.F + kWave * V - 1) / (kWave * V));
        const int cmax = max_chunks(V);
        const int sf = small_wide ? 512 : g_slice_floats;
        int C = sf > 0 ? std::max(1, sf / (kWave * V)) : cmax;
        C = std::min(C, std::min(cmax, chunks_total));
        const int slices = (chunks_total + C - 1) / C;
        const int64_t waves = n_heavy * (int64_t)C * V + n_rows;  // upper bound (VH >= 1)
        SGC_REQUIRE(waves < (int64_t)INT32_MAX, SGC_ERANGE, "spmm: too many work items");
        SGC_REQUIRE(slices < 65536, SGC_ERANGE, "spmm: too many feature slices");
        a.slices = slices;
        // the fused hub items: the 16-B-lane, one-chunk slice form (Pubmed shape)
        const bool fused = hub_deferred && V == 4 && C == 1;
        if (hub_deferred && !fused) {
            const int rc = hub_before_light();
            if (rc != SGC_OK) return rc;
        }
        if (fused) {
            a.hub_rows = hub_rows;
            a.hub_chunks = (int)((F + 31) / 32);
            a.n_hub_blocks = (int)(n_hub * a.hub_chunks);
        }
        if (timing) {
            SGC_HIP_CHECK(pooled_event(&tl.l0));
            SGC_HIP_CHECK(pooled_event(&tl.l1));
            SGC_HIP_CHECK(hipEventRecord(tl.l0, light_stream));
            tl.kernel = fused ? 3 : 0;
        }
        if (fused)
            e = launch_vc<4, 1, 32>(a);
        else if (V == 4)
            e = dispatch_c<4, max_chunks(4)>(C, a);
        else if (V == 2)
            e = dispatch_c<2, max_chunks(2)>(C, a);
        else
            e = dispatch_c<1, max_chunks(1)>(C, a);
    }
    SGC_REQUIRE(e == hipSuccess, SGC_EHIP, "spmm launch failed: %s", hipGetErrorString(e));
    if (timing) {
        SGC_HIP_CHECK(hipEventRecord(tl.l1, light_stream));
        timed_guard.commit();
    }
    if (side) SGC_HIP_CHECK(side_join.join());  // the caller's stream waits for the hub kernel
    return SGC_OK;
}

#if SGC_HUB_STAMPS
extern "C" int sgc_debug_hub_stamps(unsigned long long *host, int64_t n) {
    const int64_t cap = 5 * (int64_t)kStampRounds;
    SGC_HIP_CHECK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_hub_stamp),
                                      sizeof(unsigned long long) * (n < cap ? n : cap)));
    return SGC_OK;
}
#endif

int timing_enable(int on) {
    std::lock_guard<std::mutex> lock(g_timing_mu);
    g_timing = on != 0;
    return SGC_OK;
}

int timing_collect_ex(float *light_ms, float *hub_ms, float *span_ms, int32_t *kernel,
                      int64_t capacity, int64_t *n_host) {
    SGC_REQUIRE(n_host, SGC_EINVAL, "timing_collect: null n_host");
    std::lock_guard<std::mutex> lock(g_timing_mu);
    const int64_t n = (int64_t)g_timed.size();
    *n_host = n;
    SGC_REQUIRE(capacity >= n && (n == 0 || (light_ms && hub_ms)), SGC_ENOMEM,
                "timing_collect: capacity %lld < %lld launches", (long long)capacity,
                (long long)n);
    for (int64_t i = 0; i < n; ++i) {
        TimedLaunch &t = g_timed[(size_t)i];
        SGC_HIP_CHECK(hipEventSynchronize(t.l1));
        SGC_HIP_CHECK(hipEventElapsedTime(&light_ms[i], t.l0, t.l1));
        hub_ms[i] = -1.0f;
        float span = light_ms[i];
        if (t.h0) {
            SGC_HIP_CHECK(hipEventSynchronize(t.h1));
            SGC_HIP_CHECK(hipEventElapsedTime(&hub_ms[i], t.h0, t.h1));
            float to_end = 0.0f;
            if (t.serial) {  // h0 ... h1 l0 ... l1 on one stream
                SGC_HIP_CHECK(hipEventElapsedTime(&span, t.h0, t.l1));
            } else if (t.hub_first) {  // h0 on the caller's stream, l0 after the fork
                SGC_HIP_CHECK(hipEventElapsedTime(&to_end, t.h0, t.l1));
                span = std::max(hub_ms[i], to_end);
            }
        }
        if (span_ms) span_ms[i] = span;
        if (kernel) kernel[i] = t.kernel;
        for (hipEvent_t ev : {t.l0, t.l1, t.h0, t.h1})
            if (ev) g_event_pool.push_back(ev);
    }
    g_timed.clear();
    return SGC_OK;
}

int timing_collect(float *light_ms, float *hub_ms, int64_t capacity, int64_t *n_host) {
    return timing_collect_ex(light_ms, hub_ms, nullptr, nullptr, capacity, n_host);
}

// ---------------------------------------------------------------------------
// Row re-layout dst[i, 0:F] = src[i, 0:F]: one wave per row, V-float vectors
// (the runtime's 2-D copy blit reached only ~3 TB/s on this shape).
template <int V>
__global__ __launch_bounds__(256) void pad_rows_kernel(const float *__restrict__ src, int64_t lds,
                                                      float *__restrict__ dst, int64_t ldd,
                                                      int64_t n_rows, int F) {
    using VT = typename Vec<V>::T;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
    for (int64_t r = blockIdx.x * (int64_t)(blockDim.x / kWave) + threadIdx.x / kWave; r < n_rows;
         r += waves) {
        const VT *s = reinterpret_cast<const VT *>(src + r * lds);
        VT *d = reinterpret_cast<VT *>(dst + r * ldd);
        for (int i = lane; i < F / V; i += kWave) d[i] = s[i];
    }
}

int launch_pad_rows(const float *src, int64_t lds, float *dst, int64_t ldd, int64_t n_rows,
                    int64_t F, hipStream_t stream) {
    SGC_REQUIRE(src && dst && lds >= F && ldd >= F && n_rows >= 0 && F >= 0 && F < INT32_MAX,
                SGC_EINVAL, "pad_rows: bad arguments");
    if (n_rows == 0 || F == 0) return SGC_OK;
    const int64_t blocks = std::min<int64_t>((n_rows + 3) / 4, 256 * 16);
    const int V = pick_vec(F, lds, ldd, src, dst);
    if (V == 4)
        hipLaunchKernelGGL(pad_rows_kernel<4>, dim3(blocks), dim3(256), 0, stream, src, lds, dst,
                           ldd, n_rows, (int)F);
    else if (V == 2)
        hipLaunchKernelGGL(pad_rows_kernel<2>, dim3(blocks), dim3(256), 0, stream, src, lds, dst,
                           ldd, n_rows, (int)F);
    else
        hipLaunchKernelGGL(pad_rows_kernel<1>, dim3(blocks), dim3(256), 0, stream, src, lds, dst,
                           ldd, n_rows, (int)F);
    SGC_HIP_CHECK(hipGetLastError());
    return SGC_OK;
}

// ---------------------------------------------------------------------------
// Plan: list the rows with > threshold nonzeros, heaviest first.
__global__ void heavy_rows_kernel(const int *__restrict__ row_ptr, int row_begin, int n_rows,
                                  int threshold, int *__restrict__ out_pairs,
                                  int *__restrict__ count) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_rows;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int row = row_begin + (int)i;
        const int d = row_ptr[row + 1] - row_ptr[row];
        if (d > threshold) {
            const int pos = atomicAdd(count, 1);
            out_pairs[2 * pos] = d;
            out_pairs[2 * pos + 1] = row;
        }
    }
}

int build_plan(const int32_t *row_ptr, int64_t row_begin, int64_t row_end,
               int32_t threshold, int32_t hub_threshold, int32_t *plan, int64_t capacity,
               int64_t *n_heavy_host, int64_t *n_hub_host, hipStream_t stream) {
    SGC_REQUIRE(row_ptr && plan && n_heavy_host, SGC_EINVAL, "plan: null pointer");
    SGC_REQUIRE(hub_threshold >= threshold, SGC_EINVAL, "plan: hub_threshold < heavy_threshold");
    if (n_hub_host) *n_hub_host = 0;
    const int64_t n_rows = row_end - row_begin;
    SGC_REQUIRE(n_rows >= 0 && row_end < INT32_MAX, SGC_ERANGE, "plan: bad row range");
    SGC_REQUIRE(capacity >= 2 * n_rows + 1, SGC_ENOMEM, "plan: capacity %lld < %lld",
                (long long)capacity, (long long)(2 * n_rows + 1));
    *n_heavy_host = 0;
    if (n_rows == 0) return SGC_OK;
    int *count = plan + 2 * n_rows;  // last word is the counter
    SGC_HIP_CHECK(hipMemsetAsync(count, 0, sizeof(int), stream));
    const int blocks = (int)std::min<int64_t>((n_rows + 255) / 256, 4096);
    hipLaunchKernelGGL(heavy_rows_kernel, dim3(blocks), dim3(256), 0, stream, row_ptr,
                       (int)row_begin, (int)n_rows, threshold, plan, count);
    SGC_HIP_CHECK(hipGetLastError());
    int h = 0;
    SGC_HIP_CHECK(hipMemcpyAsync(&h, count, sizeof(int), hipMemcpyDeviceToHost, stream));
    SGC_HIP_CHECK(hipStreamSynchronize(stream));
    if (h > 0) {
        std::vector<int> pairs(2 * (size_t)h);
        SGC_HIP_CHECK(hipMemcpyAsync(pairs.data(), plan, pairs.size() * sizeof(int),
                                     hipMemcpyDeviceToHost, stream));
        SGC_HIP_CHECK(hipStreamSynchronize(stream));
        std::vector<std::pair<int, int>> dr(h);
        for (int i = 0; i < h; ++i) dr[i] = {-pairs[2 * i], pairs[2 * i + 1]};
        std::sort(dr.begin(), dr.end());  // degree desc, then row asc
        std::vector<int> rows(h);
        int64_t hubs = 0;
        for (int i = 0; i < h; ++i) {
            rows[i] = dr[i].second;
            hubs += (-dr[i].first > hub_threshold);
        }
        if (n_hub_host) *n_hub_host = hubs;
        SGC_HIP_CHECK(hipMemcpyAsync(plan, rows.data(), h * sizeof(int), hipMemcpyHostToDevice,
                                     stream));
        SGC_HIP_CHECK(hipStreamSynchronize(stream));
    }
    *n_heavy_host = h;
    return SGC_OK;
}

// Light rows (degree <= threshold) longest first, ties in row order: a
// stable counting sort over the degrees on the host (one read-back of the
// range's row_ptr through a pinned buffer; ~1 ms at Reddit shape).
int light_order(const int32_t *row_ptr, int64_t row_begin, int64_t row_end, int32_t threshold,
                int32_t *light, int64_t *n_light_host, hipStream_t stream) {
    SGC_REQUIRE(row_ptr && light && n_light_host, SGC_EINVAL, "light_order: null pointer");
    const int64_t n_rows = row_end - row_begin;
    SGC_REQUIRE(n_rows >= 0 && row_end < INT32_MAX && threshold >= 0, SGC_ERANGE,
                "light_order: bad row range or threshold");
    *n_light_host = 0;
    if (n_rows == 0) return SGC_OK;
    // pinned staging, kept for the process (grown on demand): a first large
    // pageable device-to-host copy costs the runtime tens of ms
    static std::mutex mu;
    static int32_t *pinned = nullptr;
    static size_t pinned_words = 0;
    std::lock_guard<std::mutex> lock(mu);
    const size_t need = 2 * ((size_t)n_rows + 1);  // row_ptr in, order out
    if (pinned_words < need) {
        if (pinned) SGC_HIP_CHECK(hipHostFree(pinned));
        pinned = nullptr;
        pinned_words = 0;
        SGC_HIP_CHECK(hipHostMalloc((void **)&pinned, need * sizeof(int32_t), hipHostMallocDefault));
        pinned_words = need;
    }
    int32_t *rp = pinned;
    SGC_HIP_CHECK(hipMemcpyAsync(rp, row_ptr + row_begin, ((size_t)n_rows + 1) * sizeof(int32_t),
                                 hipMemcpyDeviceToHost, stream));
    SGC_HIP_CHECK(hipStreamSynchronize(stream));
    // buckets up to the longest light row, not the threshold (which may be
    // huge: "no heavy rows")
    int64_t top = 0;
    for (int64_t i = 0; i < n_rows; ++i) {
        const int64_t d = (int64_t)rp[i + 1] - rp[i];
        if (d <= threshold && d > top) top = d;
    }
    std::vector<int64_t> start((size_t)top + 2, 0);  // bucket t = top - degree
    for (int64_t i = 0; i < n_rows; ++i) {
        const int64_t d = (int64_t)rp[i + 1] - rp[i];
        if (d <= threshold) ++start[(size_t)(top - d) + 1];
    }
    for (size_t t = 1; t < start.size(); ++t) start[t] += start[t - 1];
    const int64_t n_light = start.back();
    int32_t *out = pinned + n_rows + 1;
    for (int64_t i = 0; i < n_rows; ++i) {
        const int64_t d = (int64_t)rp[i + 1] - rp[i];
        if (d <= threshold) out[(size_t)start[(size_t)(top - d)]++] = (int32_t)(row_begin + i);
    }
    if (n_light > 0) {
        SGC_HIP_CHECK(hipMemcpyAsync(light, out, (size_t)n_light * sizeof(int32_t),
                                     hipMemcpyHostToDevice, stream));
        SGC_HIP_CHECK(hipStreamSynchronize(stream));
    }
    *n_light_host = n_light;
    return SGC_OK;
}

SGC_WARM_UNIT(warm_spmm)

hipError_t warm_side_streams() { return warm_side_streams_impl(); }

}  // namespace sgc
