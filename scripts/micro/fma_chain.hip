// Micro-benchmarks for the hub chain's floor on gfx950: cycles per step of a
// dependent v_fmac_f32 chain in ONE wave (s_memtime), fed from registers or
// from LDS in several ways.  Built and run by hand:
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/fma_chain.hip -o scripts/micro/fma_chain
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kB = 60;  // batches of 4 per round (the hub kernel's HC=64 round)

// register-only dependent chains: CH interleaved chains, 240 steps per round
template <int CH>
__global__ void reg_chain(float *out, long long *cyc, int rounds, float a, float b) {
    float acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3f + c;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int i = 0; i < 4 * kB; ++i)
#pragma unroll
            for (int c = 0; c < CH; ++c) acc[c] = __builtin_fmaf(a, acc[c], b);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// mode 0: x b128 + v b128 broadcast (the hub kernel); 1: x b128, v constant
// (SGPR); 2: x constant, v b128 broadcast; 3: x b128 + v b128, two waves'
// worth of lanes idle (HC=32: lanes 32..63 masked off)
template <int MODE>
__global__ void lds_chain(float *out, long long *cyc, int rounds, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[256];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 256; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    const f4 *xs = reinterpret_cast<const f4 *>(&x[threadIdx.x * 260]);
    const f4 *vs = reinterpret_cast<const f4 *>(v);
    float acc = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE != 3 || threadIdx.x < 32) {
        for (int r = 0; r < rounds; ++r) {
#pragma unroll
            for (int q = 0; q < kB; ++q) {
                const f4 xx = MODE == 2 ? f4{vc, vc, vc, vc} : xs[q];
                const f4 vv = MODE == 1 ? f4{vc, vc, vc, vc} : vs[q];
                acc = __builtin_fmaf(vv[0], xx[0], acc);
                acc = __builtin_fmaf(vv[1], xx[1], acc);
                acc = __builtin_fmaf(vv[2], xx[2], acc);
                acc = __builtin_fmaf(vv[3], xx[3], acc);
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    float *out;
    long long *cyc, h;
    (void)hipMalloc(&out, 1024 * 4);
    (void)hipMalloc(&cyc, 8);
    const int rounds = 2000;
    auto report = [&](const char *name, double steps) {
        (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("{\"case\": \"%s\", \"cycles_per_step\": %.2f}\n", name, (double)h / steps);
    };
#define REG(CH)                                                                          \
    for (int k = 0; k < 2; ++k)                                                          \
        hipLaunchKernelGGL(reg_chain<CH>, dim3(1), dim3(64), 0, 0, out, cyc, rounds,     \
                           1.0000001f, 1e-7f);                                           \
    report("register chain x" #CH " (per step of each chain)", rounds * 240.0);
    REG(1) REG(2) REG(4)
#define LDS(M, NAME)                                                                     \
    for (int k = 0; k < 2; ++k)                                                          \
        hipLaunchKernelGGL(lds_chain<M>, dim3(1), dim3(64), 0, 0, out, cyc, rounds, 0.5f); \
    report(NAME, rounds * 240.0);
    LDS(0, "lds: x b128 + v b128 broadcast")
    LDS(1, "lds: x b128, v in register")
    LDS(2, "lds: v b128 broadcast, x in register")
    LDS(3, "lds: x + v b128, 32 active lanes")
    int main2();
    return main2();
}

// asm rings (4 batches of LDS reads in flight, counted waits), one wave:
//  XV: x b128 + v b128 per batch (spmm_hub_kernel's chain as in hub_chain_asm)
//  X : x b128 per batch, v from an SGPR
//  XR: x b128 per batch, v by v_readlane from a VGPR (one per nonzero)
template <int MODE, int ACTIVE = 64>
__global__ void asm_chain(float *out, long long *cyc, int iters, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[256 + 64];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 256 + 64; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    uint32_t va = (uint32_t)(size_t)(lds_f *)(&v[0]);
    float acc = 0, vrow = 0.5f + threadIdx.x * 1e-3f;
    int it = iters;
    long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 0 && threadIdx.x < ACTIVE) {
        asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[80:83], %[xa]\n ds_read_b128 v[96:99], %[va]\n"
            "ds_read_b128 v[84:87], %[xa] offset:16\n ds_read_b128 v[100:103], %[va] offset:16\n"
            "ds_read_b128 v[88:91], %[xa] offset:32\n ds_read_b128 v[104:107], %[va] offset:32\n"
            "ds_read_b128 v[92:95], %[xa] offset:48\n ds_read_b128 v[108:111], %[va] offset:48\n"
            "1:\n"
            "s_waitcnt lgkmcnt(6)\n"
            "v_fmac_f32 %[acc], v96, v80\n v_fmac_f32 %[acc], v97, v81\n v_fmac_f32 %[acc], v98, v82\n v_fmac_f32 %[acc], v99, v83\n"
            "ds_read_b128 v[80:83], %[xa] offset:64\n ds_read_b128 v[96:99], %[va] offset:64\n"
            "s_waitcnt lgkmcnt(6)\n"
            "v_fmac_f32 %[acc], v100, v84\n v_fmac_f32 %[acc], v101, v85\n v_fmac_f32 %[acc], v102, v86\n v_fmac_f32 %[acc], v103, v87\n"
            "ds_read_b128 v[84:87], %[xa] offset:80\n ds_read_b128 v[100:103], %[va] offset:80\n"
            "s_waitcnt lgkmcnt(6)\n"
            "v_fmac_f32 %[acc], v104, v88\n v_fmac_f32 %[acc], v105, v89\n v_fmac_f32 %[acc], v106, v90\n v_fmac_f32 %[acc], v107, v91\n"
            "ds_read_b128 v[88:91], %[xa] offset:96\n ds_read_b128 v[104:107], %[va] offset:96\n"
            "s_waitcnt lgkmcnt(6)\n"
            "v_fmac_f32 %[acc], v108, v92\n v_fmac_f32 %[acc], v109, v93\n v_fmac_f32 %[acc], v110, v94\n v_fmac_f32 %[acc], v111, v95\n"
            "ds_read_b128 v[92:95], %[xa] offset:112\n ds_read_b128 v[108:111], %[va] offset:112\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
            : [acc] "+v"(acc), [it] "+s"(it)
            : [xa] "v"(xa), [va] "v"(va)
            : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91",
              "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102",
              "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "scc");
    } else if (MODE == 1) {
        asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[80:83], %[xa]\n"
            "ds_read_b128 v[84:87], %[xa] offset:16\n"
            "ds_read_b128 v[88:91], %[xa] offset:32\n"
            "ds_read_b128 v[92:95], %[xa] offset:48\n"
            "1:\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_fmac_f32 %[acc], %[vc], v80\n v_fmac_f32 %[acc], %[vc], v81\n v_fmac_f32 %[acc], %[vc], v82\n v_fmac_f32 %[acc], %[vc], v83\n"
            "ds_read_b128 v[80:83], %[xa] offset:64\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_fmac_f32 %[acc], %[vc], v84\n v_fmac_f32 %[acc], %[vc], v85\n v_fmac_f32 %[acc], %[vc], v86\n v_fmac_f32 %[acc], %[vc], v87\n"
            "ds_read_b128 v[84:87], %[xa] offset:80\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_fmac_f32 %[acc], %[vc], v88\n v_fmac_f32 %[acc], %[vc], v89\n v_fmac_f32 %[acc], %[vc], v90\n v_fmac_f32 %[acc], %[vc], v91\n"
            "ds_read_b128 v[88:91], %[xa] offset:96\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_fmac_f32 %[acc], %[vc], v92\n v_fmac_f32 %[acc], %[vc], v93\n v_fmac_f32 %[acc], %[vc], v94\n v_fmac_f32 %[acc], %[vc], v95\n"
            "ds_read_b128 v[92:95], %[xa] offset:112\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
            : [acc] "+v"(acc), [it] "+s"(it)
            : [xa] "v"(xa), [vc] "s"(vc)
            : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91",
              "v92", "v93", "v94", "v95", "scc");
    } else {
        asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[80:83], %[xa]\n"
            "ds_read_b128 v[84:87], %[xa] offset:16\n"
            "ds_read_b128 v[88:91], %[xa] offset:32\n"
            "ds_read_b128 v[92:95], %[xa] offset:48\n"
            "1:\n"
            "v_readlane_b32 s40, %[vr], 0\n v_readlane_b32 s41, %[vr], 1\n v_readlane_b32 s42, %[vr], 2\n v_readlane_b32 s43, %[vr], 3\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_fmac_f32 %[acc], s40, v80\n v_fmac_f32 %[acc], s41, v81\n v_fmac_f32 %[acc], s42, v82\n v_fmac_f32 %[acc], s43, v83\n"
            "ds_read_b128 v[80:83], %[xa] offset:64\n"
            "v_readlane_b32 s44, %[vr], 4\n v_readlane_b32 s45, %[vr], 5\n v_readlane_b32 s46, %[vr], 6\n v_readlane_b32 s47, %[vr], 7\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_fmac_f32 %[acc], s44, v84\n v_fmac_f32 %[acc], s45, v85\n v_fmac_f32 %[acc], s46, v86\n v_fmac_f32 %[acc], s47, v87\n"
            "ds_read_b128 v[84:87], %[xa] offset:80\n"
            "v_readlane_b32 s40, %[vr], 8\n v_readlane_b32 s41, %[vr], 9\n v_readlane_b32 s42, %[vr], 10\n v_readlane_b32 s43, %[vr], 11\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_fmac_f32 %[acc], s40, v88\n v_fmac_f32 %[acc], s41, v89\n v_fmac_f32 %[acc], s42, v90\n v_fmac_f32 %[acc], s43, v91\n"
            "ds_read_b128 v[88:91], %[xa] offset:96\n"
            "v_readlane_b32 s44, %[vr], 12\n v_readlane_b32 s45, %[vr], 13\n v_readlane_b32 s46, %[vr], 14\n v_readlane_b32 s47, %[vr], 15\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_fmac_f32 %[acc], s44, v92\n v_fmac_f32 %[acc], s45, v93\n v_fmac_f32 %[acc], s46, v94\n v_fmac_f32 %[acc], s47, v95\n"
            "ds_read_b128 v[92:95], %[xa] offset:112\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
            : [acc] "+v"(acc), [it] "+s"(it)
            : [xa] "v"(xa), [vr] "v"(vrow)
            : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91",
              "v92", "v93", "v94", "v95", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47",
              "scc");
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}


__global__ void ring_X8(float *out, long long *cyc, int iters, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[512];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    uint32_t va = (uint32_t)(size_t)(lds_f *)(&v[0]);
    float acc = 0;
    int it = iters;
    long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[80:83], %[xa] offset:0\n"
            "ds_read_b128 v[84:87], %[xa] offset:16\n"
            "ds_read_b128 v[88:91], %[xa] offset:32\n"
            "ds_read_b128 v[92:95], %[xa] offset:48\n"
            "ds_read_b128 v[96:99], %[xa] offset:64\n"
            "ds_read_b128 v[100:103], %[xa] offset:80\n"
            "ds_read_b128 v[104:107], %[xa] offset:96\n"
            "ds_read_b128 v[108:111], %[xa] offset:112\n"
            "1:\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v80\n"
            "v_fmac_f32 %[acc], %[vc], v81\n"
            "v_fmac_f32 %[acc], %[vc], v82\n"
            "v_fmac_f32 %[acc], %[vc], v83\n"
            "ds_read_b128 v[80:83], %[xa] offset:128\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v84\n"
            "v_fmac_f32 %[acc], %[vc], v85\n"
            "v_fmac_f32 %[acc], %[vc], v86\n"
            "v_fmac_f32 %[acc], %[vc], v87\n"
            "ds_read_b128 v[84:87], %[xa] offset:144\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v88\n"
            "v_fmac_f32 %[acc], %[vc], v89\n"
            "v_fmac_f32 %[acc], %[vc], v90\n"
            "v_fmac_f32 %[acc], %[vc], v91\n"
            "ds_read_b128 v[88:91], %[xa] offset:160\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v92\n"
            "v_fmac_f32 %[acc], %[vc], v93\n"
            "v_fmac_f32 %[acc], %[vc], v94\n"
            "v_fmac_f32 %[acc], %[vc], v95\n"
            "ds_read_b128 v[92:95], %[xa] offset:176\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v96\n"
            "v_fmac_f32 %[acc], %[vc], v97\n"
            "v_fmac_f32 %[acc], %[vc], v98\n"
            "v_fmac_f32 %[acc], %[vc], v99\n"
            "ds_read_b128 v[96:99], %[xa] offset:192\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v100\n"
            "v_fmac_f32 %[acc], %[vc], v101\n"
            "v_fmac_f32 %[acc], %[vc], v102\n"
            "v_fmac_f32 %[acc], %[vc], v103\n"
            "ds_read_b128 v[100:103], %[xa] offset:208\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v104\n"
            "v_fmac_f32 %[acc], %[vc], v105\n"
            "v_fmac_f32 %[acc], %[vc], v106\n"
            "v_fmac_f32 %[acc], %[vc], v107\n"
            "ds_read_b128 v[104:107], %[xa] offset:224\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v108\n"
            "v_fmac_f32 %[acc], %[vc], v109\n"
            "v_fmac_f32 %[acc], %[vc], v110\n"
            "v_fmac_f32 %[acc], %[vc], v111\n"
            "ds_read_b128 v[108:111], %[xa] offset:240\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [it] "+s"(it)
        : [xa] "v"(xa), [va] "v"(va), [vc] "s"(vc)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "scc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void ring_XV7(float *out, long long *cyc, int iters, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[512];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    uint32_t va = (uint32_t)(size_t)(lds_f *)(&v[0]);
    float acc = 0;
    int it = iters;
    long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[80:83], %[xa] offset:0\n"
            "ds_read_b128 v[108:111], %[va] offset:0\n"
            "ds_read_b128 v[84:87], %[xa] offset:16\n"
            "ds_read_b128 v[112:115], %[va] offset:16\n"
            "ds_read_b128 v[88:91], %[xa] offset:32\n"
            "ds_read_b128 v[116:119], %[va] offset:32\n"
            "ds_read_b128 v[92:95], %[xa] offset:48\n"
            "ds_read_b128 v[120:123], %[va] offset:48\n"
            "ds_read_b128 v[96:99], %[xa] offset:64\n"
            "ds_read_b128 v[124:127], %[va] offset:64\n"
            "ds_read_b128 v[100:103], %[xa] offset:80\n"
            "ds_read_b128 v[128:131], %[va] offset:80\n"
            "ds_read_b128 v[104:107], %[xa] offset:96\n"
            "ds_read_b128 v[132:135], %[va] offset:96\n"
            "1:\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v108, v80\n"
            "v_fmac_f32 %[acc], v109, v81\n"
            "v_fmac_f32 %[acc], v110, v82\n"
            "v_fmac_f32 %[acc], v111, v83\n"
            "ds_read_b128 v[80:83], %[xa] offset:112\n"
            "ds_read_b128 v[108:111], %[va] offset:112\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v112, v84\n"
            "v_fmac_f32 %[acc], v113, v85\n"
            "v_fmac_f32 %[acc], v114, v86\n"
            "v_fmac_f32 %[acc], v115, v87\n"
            "ds_read_b128 v[84:87], %[xa] offset:128\n"
            "ds_read_b128 v[112:115], %[va] offset:128\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v116, v88\n"
            "v_fmac_f32 %[acc], v117, v89\n"
            "v_fmac_f32 %[acc], v118, v90\n"
            "v_fmac_f32 %[acc], v119, v91\n"
            "ds_read_b128 v[88:91], %[xa] offset:144\n"
            "ds_read_b128 v[116:119], %[va] offset:144\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v120, v92\n"
            "v_fmac_f32 %[acc], v121, v93\n"
            "v_fmac_f32 %[acc], v122, v94\n"
            "v_fmac_f32 %[acc], v123, v95\n"
            "ds_read_b128 v[92:95], %[xa] offset:160\n"
            "ds_read_b128 v[120:123], %[va] offset:160\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v124, v96\n"
            "v_fmac_f32 %[acc], v125, v97\n"
            "v_fmac_f32 %[acc], v126, v98\n"
            "v_fmac_f32 %[acc], v127, v99\n"
            "ds_read_b128 v[96:99], %[xa] offset:176\n"
            "ds_read_b128 v[124:127], %[va] offset:176\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v128, v100\n"
            "v_fmac_f32 %[acc], v129, v101\n"
            "v_fmac_f32 %[acc], v130, v102\n"
            "v_fmac_f32 %[acc], v131, v103\n"
            "ds_read_b128 v[100:103], %[xa] offset:192\n"
            "ds_read_b128 v[128:131], %[va] offset:192\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v132, v104\n"
            "v_fmac_f32 %[acc], v133, v105\n"
            "v_fmac_f32 %[acc], v134, v106\n"
            "v_fmac_f32 %[acc], v135, v107\n"
            "ds_read_b128 v[104:107], %[xa] offset:208\n"
            "ds_read_b128 v[132:135], %[va] offset:208\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [it] "+s"(it)
        : [xa] "v"(xa), [va] "v"(va), [vc] "s"(vc)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "scc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void ring_X12(float *out, long long *cyc, int iters, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[512];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    uint32_t va = (uint32_t)(size_t)(lds_f *)(&v[0]);
    float acc = 0;
    int it = iters;
    long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[80:83], %[xa] offset:0\n"
            "ds_read_b128 v[84:87], %[xa] offset:16\n"
            "ds_read_b128 v[88:91], %[xa] offset:32\n"
            "ds_read_b128 v[92:95], %[xa] offset:48\n"
            "ds_read_b128 v[96:99], %[xa] offset:64\n"
            "ds_read_b128 v[100:103], %[xa] offset:80\n"
            "ds_read_b128 v[104:107], %[xa] offset:96\n"
            "ds_read_b128 v[108:111], %[xa] offset:112\n"
            "ds_read_b128 v[112:115], %[xa] offset:128\n"
            "ds_read_b128 v[116:119], %[xa] offset:144\n"
            "ds_read_b128 v[120:123], %[xa] offset:160\n"
            "ds_read_b128 v[124:127], %[xa] offset:176\n"
            "1:\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v80\n"
            "v_fmac_f32 %[acc], %[vc], v81\n"
            "v_fmac_f32 %[acc], %[vc], v82\n"
            "v_fmac_f32 %[acc], %[vc], v83\n"
            "ds_read_b128 v[80:83], %[xa] offset:192\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v84\n"
            "v_fmac_f32 %[acc], %[vc], v85\n"
            "v_fmac_f32 %[acc], %[vc], v86\n"
            "v_fmac_f32 %[acc], %[vc], v87\n"
            "ds_read_b128 v[84:87], %[xa] offset:208\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v88\n"
            "v_fmac_f32 %[acc], %[vc], v89\n"
            "v_fmac_f32 %[acc], %[vc], v90\n"
            "v_fmac_f32 %[acc], %[vc], v91\n"
            "ds_read_b128 v[88:91], %[xa] offset:224\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v92\n"
            "v_fmac_f32 %[acc], %[vc], v93\n"
            "v_fmac_f32 %[acc], %[vc], v94\n"
            "v_fmac_f32 %[acc], %[vc], v95\n"
            "ds_read_b128 v[92:95], %[xa] offset:240\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v96\n"
            "v_fmac_f32 %[acc], %[vc], v97\n"
            "v_fmac_f32 %[acc], %[vc], v98\n"
            "v_fmac_f32 %[acc], %[vc], v99\n"
            "ds_read_b128 v[96:99], %[xa] offset:256\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v100\n"
            "v_fmac_f32 %[acc], %[vc], v101\n"
            "v_fmac_f32 %[acc], %[vc], v102\n"
            "v_fmac_f32 %[acc], %[vc], v103\n"
            "ds_read_b128 v[100:103], %[xa] offset:272\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v104\n"
            "v_fmac_f32 %[acc], %[vc], v105\n"
            "v_fmac_f32 %[acc], %[vc], v106\n"
            "v_fmac_f32 %[acc], %[vc], v107\n"
            "ds_read_b128 v[104:107], %[xa] offset:288\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v108\n"
            "v_fmac_f32 %[acc], %[vc], v109\n"
            "v_fmac_f32 %[acc], %[vc], v110\n"
            "v_fmac_f32 %[acc], %[vc], v111\n"
            "ds_read_b128 v[108:111], %[xa] offset:304\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v112\n"
            "v_fmac_f32 %[acc], %[vc], v113\n"
            "v_fmac_f32 %[acc], %[vc], v114\n"
            "v_fmac_f32 %[acc], %[vc], v115\n"
            "ds_read_b128 v[112:115], %[xa] offset:320\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v116\n"
            "v_fmac_f32 %[acc], %[vc], v117\n"
            "v_fmac_f32 %[acc], %[vc], v118\n"
            "v_fmac_f32 %[acc], %[vc], v119\n"
            "ds_read_b128 v[116:119], %[xa] offset:336\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v120\n"
            "v_fmac_f32 %[acc], %[vc], v121\n"
            "v_fmac_f32 %[acc], %[vc], v122\n"
            "v_fmac_f32 %[acc], %[vc], v123\n"
            "ds_read_b128 v[120:123], %[xa] offset:352\n"
            "s_waitcnt lgkmcnt(11)\n"
            "v_fmac_f32 %[acc], %[vc], v124\n"
            "v_fmac_f32 %[acc], %[vc], v125\n"
            "v_fmac_f32 %[acc], %[vc], v126\n"
            "v_fmac_f32 %[acc], %[vc], v127\n"
            "ds_read_b128 v[124:127], %[xa] offset:368\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [it] "+s"(it)
        : [xa] "v"(xa), [va] "v"(va), [vc] "s"(vc)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "scc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}


__global__ void ring_B64x8(float *out, long long *cyc, int iters, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[512];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    uint32_t va = (uint32_t)(size_t)(lds_f *)(&v[0]);
    float acc = 0;
    int it = iters;
    long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b64 v[80:81], %[xa] offset:0\n"
            "ds_read_b64 v[82:83], %[xa] offset:8\n"
            "ds_read_b64 v[84:85], %[xa] offset:16\n"
            "ds_read_b64 v[86:87], %[xa] offset:24\n"
            "ds_read_b64 v[88:89], %[xa] offset:32\n"
            "ds_read_b64 v[90:91], %[xa] offset:40\n"
            "ds_read_b64 v[92:93], %[xa] offset:48\n"
            "ds_read_b64 v[94:95], %[xa] offset:56\n"
            "1:\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v80\n"
            "v_fmac_f32 %[acc], %[vc], v81\n"
            "ds_read_b64 v[80:81], %[xa] offset:64\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v82\n"
            "v_fmac_f32 %[acc], %[vc], v83\n"
            "ds_read_b64 v[82:83], %[xa] offset:72\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v84\n"
            "v_fmac_f32 %[acc], %[vc], v85\n"
            "ds_read_b64 v[84:85], %[xa] offset:80\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v86\n"
            "v_fmac_f32 %[acc], %[vc], v87\n"
            "ds_read_b64 v[86:87], %[xa] offset:88\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v88\n"
            "v_fmac_f32 %[acc], %[vc], v89\n"
            "ds_read_b64 v[88:89], %[xa] offset:96\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v90\n"
            "v_fmac_f32 %[acc], %[vc], v91\n"
            "ds_read_b64 v[90:91], %[xa] offset:104\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v92\n"
            "v_fmac_f32 %[acc], %[vc], v93\n"
            "ds_read_b64 v[92:93], %[xa] offset:112\n"
            "s_waitcnt lgkmcnt(7)\n"
            "v_fmac_f32 %[acc], %[vc], v94\n"
            "v_fmac_f32 %[acc], %[vc], v95\n"
            "ds_read_b64 v[94:95], %[xa] offset:120\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [it] "+s"(it)
        : [xa] "v"(xa), [va] "v"(va), [vc] "s"(vc)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "scc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void ring_B64x14(float *out, long long *cyc, int iters, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[512];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    uint32_t va = (uint32_t)(size_t)(lds_f *)(&v[0]);
    float acc = 0;
    int it = iters;
    long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b64 v[80:81], %[xa] offset:0\n"
            "ds_read_b64 v[82:83], %[xa] offset:8\n"
            "ds_read_b64 v[84:85], %[xa] offset:16\n"
            "ds_read_b64 v[86:87], %[xa] offset:24\n"
            "ds_read_b64 v[88:89], %[xa] offset:32\n"
            "ds_read_b64 v[90:91], %[xa] offset:40\n"
            "ds_read_b64 v[92:93], %[xa] offset:48\n"
            "ds_read_b64 v[94:95], %[xa] offset:56\n"
            "ds_read_b64 v[96:97], %[xa] offset:64\n"
            "ds_read_b64 v[98:99], %[xa] offset:72\n"
            "ds_read_b64 v[100:101], %[xa] offset:80\n"
            "ds_read_b64 v[102:103], %[xa] offset:88\n"
            "ds_read_b64 v[104:105], %[xa] offset:96\n"
            "ds_read_b64 v[106:107], %[xa] offset:104\n"
            "1:\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v80\n"
            "v_fmac_f32 %[acc], %[vc], v81\n"
            "ds_read_b64 v[80:81], %[xa] offset:112\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v82\n"
            "v_fmac_f32 %[acc], %[vc], v83\n"
            "ds_read_b64 v[82:83], %[xa] offset:120\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v84\n"
            "v_fmac_f32 %[acc], %[vc], v85\n"
            "ds_read_b64 v[84:85], %[xa] offset:128\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v86\n"
            "v_fmac_f32 %[acc], %[vc], v87\n"
            "ds_read_b64 v[86:87], %[xa] offset:136\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v88\n"
            "v_fmac_f32 %[acc], %[vc], v89\n"
            "ds_read_b64 v[88:89], %[xa] offset:144\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v90\n"
            "v_fmac_f32 %[acc], %[vc], v91\n"
            "ds_read_b64 v[90:91], %[xa] offset:152\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v92\n"
            "v_fmac_f32 %[acc], %[vc], v93\n"
            "ds_read_b64 v[92:93], %[xa] offset:160\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v94\n"
            "v_fmac_f32 %[acc], %[vc], v95\n"
            "ds_read_b64 v[94:95], %[xa] offset:168\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v96\n"
            "v_fmac_f32 %[acc], %[vc], v97\n"
            "ds_read_b64 v[96:97], %[xa] offset:176\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v98\n"
            "v_fmac_f32 %[acc], %[vc], v99\n"
            "ds_read_b64 v[98:99], %[xa] offset:184\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v100\n"
            "v_fmac_f32 %[acc], %[vc], v101\n"
            "ds_read_b64 v[100:101], %[xa] offset:192\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v102\n"
            "v_fmac_f32 %[acc], %[vc], v103\n"
            "ds_read_b64 v[102:103], %[xa] offset:200\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v104\n"
            "v_fmac_f32 %[acc], %[vc], v105\n"
            "ds_read_b64 v[104:105], %[xa] offset:208\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v106\n"
            "v_fmac_f32 %[acc], %[vc], v107\n"
            "ds_read_b64 v[106:107], %[xa] offset:216\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [it] "+s"(it)
        : [xa] "v"(xa), [va] "v"(va), [vc] "s"(vc)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "scc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void ring_B32x14(float *out, long long *cyc, int iters, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[512];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    uint32_t va = (uint32_t)(size_t)(lds_f *)(&v[0]);
    float acc = 0;
    int it = iters;
    long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b32 v80, %[xa] offset:0\n"
            "ds_read_b32 v81, %[xa] offset:4\n"
            "ds_read_b32 v82, %[xa] offset:8\n"
            "ds_read_b32 v83, %[xa] offset:12\n"
            "ds_read_b32 v84, %[xa] offset:16\n"
            "ds_read_b32 v85, %[xa] offset:20\n"
            "ds_read_b32 v86, %[xa] offset:24\n"
            "ds_read_b32 v87, %[xa] offset:28\n"
            "ds_read_b32 v88, %[xa] offset:32\n"
            "ds_read_b32 v89, %[xa] offset:36\n"
            "ds_read_b32 v90, %[xa] offset:40\n"
            "ds_read_b32 v91, %[xa] offset:44\n"
            "ds_read_b32 v92, %[xa] offset:48\n"
            "ds_read_b32 v93, %[xa] offset:52\n"
            "1:\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v80\n"
            "ds_read_b32 v80, %[xa] offset:56\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v81\n"
            "ds_read_b32 v81, %[xa] offset:60\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v82\n"
            "ds_read_b32 v82, %[xa] offset:64\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v83\n"
            "ds_read_b32 v83, %[xa] offset:68\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v84\n"
            "ds_read_b32 v84, %[xa] offset:72\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v85\n"
            "ds_read_b32 v85, %[xa] offset:76\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v86\n"
            "ds_read_b32 v86, %[xa] offset:80\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v87\n"
            "ds_read_b32 v87, %[xa] offset:84\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v88\n"
            "ds_read_b32 v88, %[xa] offset:88\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v89\n"
            "ds_read_b32 v89, %[xa] offset:92\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v90\n"
            "ds_read_b32 v90, %[xa] offset:96\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v91\n"
            "ds_read_b32 v91, %[xa] offset:100\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v92\n"
            "ds_read_b32 v92, %[xa] offset:104\n"
            "s_waitcnt lgkmcnt(13)\n"
            "v_fmac_f32 %[acc], %[vc], v93\n"
            "ds_read_b32 v93, %[xa] offset:108\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [it] "+s"(it)
        : [xa] "v"(xa), [va] "v"(va), [vc] "s"(vc)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "scc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void ring_B64V7(float *out, long long *cyc, int iters, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[512];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    uint32_t va = (uint32_t)(size_t)(lds_f *)(&v[0]);
    float acc = 0;
    int it = iters;
    long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b64 v[80:81], %[xa] offset:0\n"
            "ds_read_b64 v[94:95], %[va] offset:0\n"
            "ds_read_b64 v[82:83], %[xa] offset:8\n"
            "ds_read_b64 v[96:97], %[va] offset:8\n"
            "ds_read_b64 v[84:85], %[xa] offset:16\n"
            "ds_read_b64 v[98:99], %[va] offset:16\n"
            "ds_read_b64 v[86:87], %[xa] offset:24\n"
            "ds_read_b64 v[100:101], %[va] offset:24\n"
            "ds_read_b64 v[88:89], %[xa] offset:32\n"
            "ds_read_b64 v[102:103], %[va] offset:32\n"
            "ds_read_b64 v[90:91], %[xa] offset:40\n"
            "ds_read_b64 v[104:105], %[va] offset:40\n"
            "ds_read_b64 v[92:93], %[xa] offset:48\n"
            "ds_read_b64 v[106:107], %[va] offset:48\n"
            "1:\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v94, v80\n"
            "v_fmac_f32 %[acc], v95, v81\n"
            "ds_read_b64 v[80:81], %[xa] offset:56\n"
            "ds_read_b64 v[94:95], %[va] offset:56\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v96, v82\n"
            "v_fmac_f32 %[acc], v97, v83\n"
            "ds_read_b64 v[82:83], %[xa] offset:64\n"
            "ds_read_b64 v[96:97], %[va] offset:64\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v98, v84\n"
            "v_fmac_f32 %[acc], v99, v85\n"
            "ds_read_b64 v[84:85], %[xa] offset:72\n"
            "ds_read_b64 v[98:99], %[va] offset:72\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v100, v86\n"
            "v_fmac_f32 %[acc], v101, v87\n"
            "ds_read_b64 v[86:87], %[xa] offset:80\n"
            "ds_read_b64 v[100:101], %[va] offset:80\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v102, v88\n"
            "v_fmac_f32 %[acc], v103, v89\n"
            "ds_read_b64 v[88:89], %[xa] offset:88\n"
            "ds_read_b64 v[102:103], %[va] offset:88\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v104, v90\n"
            "v_fmac_f32 %[acc], v105, v91\n"
            "ds_read_b64 v[90:91], %[xa] offset:96\n"
            "ds_read_b64 v[104:105], %[va] offset:96\n"
            "s_waitcnt lgkmcnt(12)\n"
            "v_fmac_f32 %[acc], v106, v92\n"
            "v_fmac_f32 %[acc], v107, v93\n"
            "ds_read_b64 v[92:93], %[xa] offset:104\n"
            "ds_read_b64 v[106:107], %[va] offset:104\n"
            "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [it] "+s"(it)
        : [xa] "v"(xa), [va] "v"(va), [vc] "s"(vc)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "scc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}


// v values by scalar buffer loads (three 16-value SGPR banks, loaded two
// chunks ahead, streaming through a 2 MB buffer: scalar-cache misses), x by
// ds_read_b128 (the next 16 nonzeros' half while this half's FMAs run); one
// lgkmcnt(0) per 16 nonzeros (scalar loads complete out of order).
__global__ void ring_XS(float *out, long long *cyc, int iters, const float *vals) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    typedef int i4 __attribute__((ext_vector_type(4)));
    const uint64_t base = (uint64_t)vals;
    i4 rs;
    rs[0] = __builtin_amdgcn_readfirstlane((int)(base & 0xffffffffu));
    rs[1] = __builtin_amdgcn_readfirstlane((int)(base >> 32));
    rs[2] = 0x200000;  // num_records (bytes)
    rs[3] = 0x00020000;
    uint32_t vo = 0;
    float acc = 0;
    int it = iters;
    long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
            "s_waitcnt lgkmcnt(0)\n"
            "s_buffer_load_dwordx16 s[40:55], %[rs], %[vo]\n"
            "s_add_u32 %[vo], %[vo], 64\n"
            "s_buffer_load_dwordx16 s[56:71], %[rs], %[vo]\n"
            "s_add_u32 %[vo], %[vo], 64\n"
            "ds_read_b128 v[80:83], %[xa] offset:0\n"
            "ds_read_b128 v[84:87], %[xa] offset:16\n"
            "ds_read_b128 v[88:91], %[xa] offset:32\n"
            "ds_read_b128 v[92:95], %[xa] offset:48\n"
            "s_waitcnt lgkmcnt(0)\n"
            "1:\n"
            "ds_read_b128 v[96:99], %[xa] offset:64\n"
            "ds_read_b128 v[100:103], %[xa] offset:80\n"
            "ds_read_b128 v[104:107], %[xa] offset:96\n"
            "ds_read_b128 v[108:111], %[xa] offset:112\n"
            "s_buffer_load_dwordx16 s[72:87], %[rs], %[vo]\n"
            "s_add_u32 %[vo], %[vo], 64\n"
            "s_and_b32 %[vo], %[vo], 0x1fffff\n"
            "v_fmac_f32 %[acc], s40, v80\n"
            "v_fmac_f32 %[acc], s41, v81\n"
            "v_fmac_f32 %[acc], s42, v82\n"
            "v_fmac_f32 %[acc], s43, v83\n"
            "v_fmac_f32 %[acc], s44, v84\n"
            "v_fmac_f32 %[acc], s45, v85\n"
            "v_fmac_f32 %[acc], s46, v86\n"
            "v_fmac_f32 %[acc], s47, v87\n"
            "v_fmac_f32 %[acc], s48, v88\n"
            "v_fmac_f32 %[acc], s49, v89\n"
            "v_fmac_f32 %[acc], s50, v90\n"
            "v_fmac_f32 %[acc], s51, v91\n"
            "v_fmac_f32 %[acc], s52, v92\n"
            "v_fmac_f32 %[acc], s53, v93\n"
            "v_fmac_f32 %[acc], s54, v94\n"
            "v_fmac_f32 %[acc], s55, v95\n"
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[80:83], %[xa] offset:64\n"
            "ds_read_b128 v[84:87], %[xa] offset:80\n"
            "ds_read_b128 v[88:91], %[xa] offset:96\n"
            "ds_read_b128 v[92:95], %[xa] offset:112\n"
            "s_buffer_load_dwordx16 s[40:55], %[rs], %[vo]\n"
            "s_add_u32 %[vo], %[vo], 64\n"
            "s_and_b32 %[vo], %[vo], 0x1fffff\n"
            "v_fmac_f32 %[acc], s56, v96\n"
            "v_fmac_f32 %[acc], s57, v97\n"
            "v_fmac_f32 %[acc], s58, v98\n"
            "v_fmac_f32 %[acc], s59, v99\n"
            "v_fmac_f32 %[acc], s60, v100\n"
            "v_fmac_f32 %[acc], s61, v101\n"
            "v_fmac_f32 %[acc], s62, v102\n"
            "v_fmac_f32 %[acc], s63, v103\n"
            "v_fmac_f32 %[acc], s64, v104\n"
            "v_fmac_f32 %[acc], s65, v105\n"
            "v_fmac_f32 %[acc], s66, v106\n"
            "v_fmac_f32 %[acc], s67, v107\n"
            "v_fmac_f32 %[acc], s68, v108\n"
            "v_fmac_f32 %[acc], s69, v109\n"
            "v_fmac_f32 %[acc], s70, v110\n"
            "v_fmac_f32 %[acc], s71, v111\n"
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[96:99], %[xa] offset:64\n"
            "ds_read_b128 v[100:103], %[xa] offset:80\n"
            "ds_read_b128 v[104:107], %[xa] offset:96\n"
            "ds_read_b128 v[108:111], %[xa] offset:112\n"
            "s_buffer_load_dwordx16 s[56:71], %[rs], %[vo]\n"
            "s_add_u32 %[vo], %[vo], 64\n"
            "s_and_b32 %[vo], %[vo], 0x1fffff\n"
            "v_fmac_f32 %[acc], s72, v80\n"
            "v_fmac_f32 %[acc], s73, v81\n"
            "v_fmac_f32 %[acc], s74, v82\n"
            "v_fmac_f32 %[acc], s75, v83\n"
            "v_fmac_f32 %[acc], s76, v84\n"
            "v_fmac_f32 %[acc], s77, v85\n"
            "v_fmac_f32 %[acc], s78, v86\n"
            "v_fmac_f32 %[acc], s79, v87\n"
            "v_fmac_f32 %[acc], s80, v88\n"
            "v_fmac_f32 %[acc], s81, v89\n"
            "v_fmac_f32 %[acc], s82, v90\n"
            "v_fmac_f32 %[acc], s83, v91\n"
            "v_fmac_f32 %[acc], s84, v92\n"
            "v_fmac_f32 %[acc], s85, v93\n"
            "v_fmac_f32 %[acc], s86, v94\n"
            "v_fmac_f32 %[acc], s87, v95\n"
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[80:83], %[xa] offset:64\n"
            "ds_read_b128 v[84:87], %[xa] offset:80\n"
            "ds_read_b128 v[88:91], %[xa] offset:96\n"
            "ds_read_b128 v[92:95], %[xa] offset:112\n"
            "s_buffer_load_dwordx16 s[72:87], %[rs], %[vo]\n"
            "s_add_u32 %[vo], %[vo], 64\n"
            "s_and_b32 %[vo], %[vo], 0x1fffff\n"
            "v_fmac_f32 %[acc], s40, v96\n"
            "v_fmac_f32 %[acc], s41, v97\n"
            "v_fmac_f32 %[acc], s42, v98\n"
            "v_fmac_f32 %[acc], s43, v99\n"
            "v_fmac_f32 %[acc], s44, v100\n"
            "v_fmac_f32 %[acc], s45, v101\n"
            "v_fmac_f32 %[acc], s46, v102\n"
            "v_fmac_f32 %[acc], s47, v103\n"
            "v_fmac_f32 %[acc], s48, v104\n"
            "v_fmac_f32 %[acc], s49, v105\n"
            "v_fmac_f32 %[acc], s50, v106\n"
            "v_fmac_f32 %[acc], s51, v107\n"
            "v_fmac_f32 %[acc], s52, v108\n"
            "v_fmac_f32 %[acc], s53, v109\n"
            "v_fmac_f32 %[acc], s54, v110\n"
            "v_fmac_f32 %[acc], s55, v111\n"
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[96:99], %[xa] offset:64\n"
            "ds_read_b128 v[100:103], %[xa] offset:80\n"
            "ds_read_b128 v[104:107], %[xa] offset:96\n"
            "ds_read_b128 v[108:111], %[xa] offset:112\n"
            "s_buffer_load_dwordx16 s[40:55], %[rs], %[vo]\n"
            "s_add_u32 %[vo], %[vo], 64\n"
            "s_and_b32 %[vo], %[vo], 0x1fffff\n"
            "v_fmac_f32 %[acc], s56, v80\n"
            "v_fmac_f32 %[acc], s57, v81\n"
            "v_fmac_f32 %[acc], s58, v82\n"
            "v_fmac_f32 %[acc], s59, v83\n"
            "v_fmac_f32 %[acc], s60, v84\n"
            "v_fmac_f32 %[acc], s61, v85\n"
            "v_fmac_f32 %[acc], s62, v86\n"
            "v_fmac_f32 %[acc], s63, v87\n"
            "v_fmac_f32 %[acc], s64, v88\n"
            "v_fmac_f32 %[acc], s65, v89\n"
            "v_fmac_f32 %[acc], s66, v90\n"
            "v_fmac_f32 %[acc], s67, v91\n"
            "v_fmac_f32 %[acc], s68, v92\n"
            "v_fmac_f32 %[acc], s69, v93\n"
            "v_fmac_f32 %[acc], s70, v94\n"
            "v_fmac_f32 %[acc], s71, v95\n"
            "s_waitcnt lgkmcnt(0)\n"
            "ds_read_b128 v[80:83], %[xa] offset:64\n"
            "ds_read_b128 v[84:87], %[xa] offset:80\n"
            "ds_read_b128 v[88:91], %[xa] offset:96\n"
            "ds_read_b128 v[92:95], %[xa] offset:112\n"
            "s_buffer_load_dwordx16 s[56:71], %[rs], %[vo]\n"
            "s_add_u32 %[vo], %[vo], 64\n"
            "s_and_b32 %[vo], %[vo], 0x1fffff\n"
            "v_fmac_f32 %[acc], s72, v96\n"
            "v_fmac_f32 %[acc], s73, v97\n"
            "v_fmac_f32 %[acc], s74, v98\n"
            "v_fmac_f32 %[acc], s75, v99\n"
            "v_fmac_f32 %[acc], s76, v100\n"
            "v_fmac_f32 %[acc], s77, v101\n"
            "v_fmac_f32 %[acc], s78, v102\n"
            "v_fmac_f32 %[acc], s79, v103\n"
            "v_fmac_f32 %[acc], s80, v104\n"
            "v_fmac_f32 %[acc], s81, v105\n"
            "v_fmac_f32 %[acc], s82, v106\n"
            "v_fmac_f32 %[acc], s83, v107\n"
            "v_fmac_f32 %[acc], s84, v108\n"
            "v_fmac_f32 %[acc], s85, v109\n"
            "v_fmac_f32 %[acc], s86, v110\n"
            "v_fmac_f32 %[acc], s87, v111\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_sub_u32 %[it], %[it], 1\n"
            "s_cmp_lg_u32 %[it], 0\n"
            "s_cbranch_scc1 1b\n"
            "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [it] "+s"(it), [vo] "+s"(vo)
        : [xa] "v"(xa), [rs] "s"(rs)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "scc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// S values off the LDS-read path by DPP: one ds_read_b32 per 16 nonzeros
// (lane l holds v[l & 15], so every 16-lane row has all 16) and each FMA
// broadcasts lane k of its row with row_newbcast:k; X as in ring_X8 (b128
// ring, 8 batches = 2 iterations ahead).  Same FMA order and operands as the
// hub chain: acc = fma(v[k], x[k], acc).
__global__ void ring_XDPP(float *out, long long *cyc, int iters, float vc) {
    __shared__ __attribute__((aligned(16))) float x[64 * 260];
    __shared__ __attribute__((aligned(16))) float v[512];
    for (int i = threadIdx.x; i < 64 * 260; i += blockDim.x) x[i] = 1e-3f * (i % 97);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) v[i] = 0.5f + 1e-3f * i;
    __syncthreads();
    typedef __attribute__((address_space(3))) const float lds_f;
    uint32_t xa = (uint32_t)(size_t)(lds_f *)(&x[threadIdx.x * 260]);
    uint32_t vl = (uint32_t)(size_t)(lds_f *)(&v[threadIdx.x & 15]);
    float acc = 0;
    int it = iters;
    (void)vc;
    long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n"
        "ds_read_b32 v112, %[vl] offset:0\n"
        "ds_read_b128 v[80:83], %[xa] offset:0\n"
        "ds_read_b128 v[84:87], %[xa] offset:16\n"
        "ds_read_b128 v[88:91], %[xa] offset:32\n"
        "ds_read_b128 v[92:95], %[xa] offset:48\n"
        "ds_read_b32 v113, %[vl] offset:64\n"
        "ds_read_b128 v[96:99], %[xa] offset:64\n"
        "ds_read_b128 v[100:103], %[xa] offset:80\n"
        "ds_read_b128 v[104:107], %[xa] offset:96\n"
        "ds_read_b128 v[108:111], %[xa] offset:112\n"
        "1:\n"
        // iteration A: v112, slots v80..v95
        "s_waitcnt lgkmcnt(8)\n"
        "v_fmac_f32_dpp %[acc], v112, v80 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v81 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v82 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v83 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[80:83], %[xa] offset:128\n"
        "s_waitcnt lgkmcnt(8)\n"
        "v_fmac_f32_dpp %[acc], v112, v84 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v85 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v86 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v87 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[84:87], %[xa] offset:144\n"
        "s_waitcnt lgkmcnt(8)\n"
        "v_fmac_f32_dpp %[acc], v112, v88 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v89 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v90 row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v91 row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[88:91], %[xa] offset:160\n"
        "s_waitcnt lgkmcnt(8)\n"
        "v_fmac_f32_dpp %[acc], v112, v92 row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v93 row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v94 row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v112, v95 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[92:95], %[xa] offset:176\n"
        "ds_read_b32 v112, %[vl] offset:128\n"
        // iteration B: v113, slots v96..v111
        "s_waitcnt lgkmcnt(8)\n"
        "v_fmac_f32_dpp %[acc], v113, v96 row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v97 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v98 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v99 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[96:99], %[xa] offset:192\n"
        "s_waitcnt lgkmcnt(8)\n"
        "v_fmac_f32_dpp %[acc], v113, v100 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v101 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v102 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v103 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[100:103], %[xa] offset:208\n"
        "s_waitcnt lgkmcnt(8)\n"
        "v_fmac_f32_dpp %[acc], v113, v104 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v105 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v106 row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v107 row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[104:107], %[xa] offset:224\n"
        "s_waitcnt lgkmcnt(8)\n"
        "v_fmac_f32_dpp %[acc], v113, v108 row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v109 row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v110 row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f32_dpp %[acc], v113, v111 row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "ds_read_b128 v[108:111], %[xa] offset:240\n"
        "ds_read_b32 v113, %[vl] offset:192\n"
        "s_sub_u32 %[it], %[it], 1\n s_cmp_lg_u32 %[it], 0\n s_cbranch_scc1 1b\n"
        "s_waitcnt lgkmcnt(0)\n"
        : [acc] "+v"(acc), [it] "+s"(it)
        : [xa] "v"(xa), [vl] "v"(vl)
        : "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91",
          "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102",
          "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112",
          "v113", "scc");
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main6() {
    float *out;
    long long *cyc, h;
    (void)hipMalloc(&out, 1024 * 4);
    (void)hipMalloc(&cyc, 8);
    const int iters = 20000;  // x 32 nonzeros
    for (int k = 0; k < 2; ++k)
        hipLaunchKernelGGL(ring_XDPP, dim3(1), dim3(64), 0, 0, out, cyc, iters, 0.5f);
    (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"case\": \"%s\", \"cycles_per_nonzero\": %.2f}\n",
           "asm ring 8 batches: x b128, v by ds_read_b32 per 16 + DPP row_newbcast",
           (double)h / (iters * 32.0));
    return 0;
}

int main5() {
    float *out, *vals;
    long long *cyc, h;
    (void)hipMalloc(&out, 1024 * 4);
    (void)hipMalloc(&cyc, 8);
    (void)hipMalloc(&vals, 0x200000);
    (void)hipMemset(vals, 0, 0x200000);
    const int iters = 20000;  // x 6 x 16 nonzeros
    for (int k = 0; k < 2; ++k)
        hipLaunchKernelGGL(ring_XS, dim3(1), dim3(64), 0, 0, out, cyc, iters, (const float *)vals);
    (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"case\": \"%s\", \"cycles_per_nonzero\": %.2f}\n",
           "x b128 half-ring + v by s_buffer_load_dwordx16 (3 banks, 2 ahead)",
           (double)h / (iters * 96.0));
    return main6();
}

int main4() {
    float *out;
    long long *cyc, h;
    (void)hipMalloc(&out, 1024 * 4);
    (void)hipMalloc(&cyc, 8);
    const int iters = 20000;
#define RUN4(K, NNZ, NAME)                                                                   \
    for (int k = 0; k < 2; ++k)                                                              \
        hipLaunchKernelGGL(K, dim3(1), dim3(64), 0, 0, out, cyc, iters, 0.5f);               \
    (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);                                      \
    printf("{\"case\": \"%s\", \"cycles_per_nonzero\": %.2f}\n", NAME, (double)h / (iters * (double)(NNZ)));
    RUN4(ring_B64x8, 16, "asm ring 8 x ds_read_b64 (2 nnz each), v in SGPR")
    RUN4(ring_B64x14, 28, "asm ring 14 x ds_read_b64, v in SGPR")
    RUN4(ring_B32x14, 14, "asm ring 14 x ds_read_b32, v in SGPR")
    RUN4(ring_B64V7, 14, "asm ring 7 x (x ds_read_b64 + v ds_read_b64)")
    return main5();
}

int main3() {
    float *out;
    long long *cyc, h;
    (void)hipMalloc(&out, 1024 * 4);
    (void)hipMalloc(&cyc, 8);
    const int iters = 20000;
#define RUN(K, D, NAME)                                                                      \
    for (int k = 0; k < 2; ++k)                                                              \
        hipLaunchKernelGGL(K, dim3(1), dim3(64), 0, 0, out, cyc, iters, 0.5f);               \
    (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);                                      \
    printf("{\"case\": \"%s\", \"cycles_per_nonzero\": %.2f}\n", NAME, (double)h / (iters * 4.0 * D));
    RUN(ring_X8, 8, "asm ring 8 batches: x b128, v in SGPR")
    RUN(ring_XV7, 7, "asm ring 7 batches: x b128 + v b128")
    RUN(ring_X12, 12, "asm ring 12 batches: x b128, v in SGPR")
    return main4();
}

int main2() {
    float *out;
    long long *cyc, h;
    (void)hipMalloc(&out, 1024 * 4);
    (void)hipMalloc(&cyc, 8);
    const int iters = 20000;  // x 16 nonzeros (reads stay inside the image: offsets repeat)
    const char *names[5] = {"asm ring: x b128 + v b128", "asm ring: x b128, v in SGPR",
                            "asm ring: x b128, v by v_readlane", "asm ring: x+v, 32 lanes active",
                            "asm ring: x+v, 16 lanes active"};
    for (int m = 0; m < 5; ++m) {
        for (int k = 0; k < 2; ++k) {
            if (m == 0) hipLaunchKernelGGL(asm_chain<0>, dim3(1), dim3(64), 0, 0, out, cyc, iters, 0.5f);
            if (m == 1) hipLaunchKernelGGL(asm_chain<1>, dim3(1), dim3(64), 0, 0, out, cyc, iters, 0.5f);
            if (m == 2) hipLaunchKernelGGL(asm_chain<2>, dim3(1), dim3(64), 0, 0, out, cyc, iters, 0.5f);
            if (m == 3) hipLaunchKernelGGL((asm_chain<0, 32>), dim3(1), dim3(64), 0, 0, out, cyc, iters, 0.5f);
            if (m == 4) hipLaunchKernelGGL((asm_chain<0, 16>), dim3(1), dim3(64), 0, 0, out, cyc, iters, 0.5f);
        }
        (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("{\"case\": \"%s\", \"cycles_per_nonzero\": %.2f}\n", names[m], (double)h / (iters * 16.0));
    }
    return main3();
}
