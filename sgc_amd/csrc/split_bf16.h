// split_bf16.h -- exact three-piece bf16 split of fp32 operands (the
// classifier's MFMA kernels, linear.hip and xent.hip): x = h + m + l with
// h = RNE(x), m = RNE(x - h), l = x - h - m (each difference exact by
// Sterbenz), so x . w on v_mfma_f32_16x16x32_bf16 as the six products hh,
// hm, mh, hl, lh, mm reaches fp32 precision (the dropped ml, lm, ll are below
// 2^-25 of |x||w|).  Finite values only (x - h is inf - inf for infinite x).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sgc {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    const bf16x2_t v = {(__bf16)a, (__bf16)b};  // v_cvt_pk_bf16_f32 (RNE)
    return __builtin_bit_cast(uint32_t, v);
}

// (a, b) -> packed hi / mid / lo bf16 pairs with a == hi + mid + lo exactly
// (finite a, b).
__device__ __forceinline__ void split3(float a, float b, uint32_t &h, uint32_t &m, uint32_t &l) {
    h = pk_bf16(a, b);
    const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xffff0000u);
    m = pk_bf16(ra, rb);
    l = pk_bf16(ra - __uint_as_float(m << 16), rb - __uint_as_float(m & 0xffff0000u));
}

}  // namespace sgc
