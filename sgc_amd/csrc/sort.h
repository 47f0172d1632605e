// sort.h -- the library's own stable radix sort (sort.hip).
#pragma once

#include "common.h"

namespace sgc {

// Bytes of device workspace radix_sort_pairs needs for n pairs.
int64_t radix_sort_workspace(int64_t n);

// Stable LSD radix sort of n (key, value) pairs by key: ascending, or
// descending when `descending` (keys compared as key_max - key, so ties keep
// their input order either way).  Every key must be <= key_max; the number of
// 11-bit passes follows key_max.  keys_out / vals_out must not alias the
// inputs.  Asynchronous on `stream`; no host synchronisation.
int radix_sort_pairs(const uint32_t *keys_in, const int32_t *vals_in, uint32_t *keys_out,
                     int32_t *vals_out, int64_t n, uint32_t key_max, bool descending, void *ws,
                     int64_t ws_bytes, hipStream_t stream);

}  // namespace sgc
