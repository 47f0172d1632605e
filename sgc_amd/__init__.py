"""sgc_amd -- MI355X-native (gfx950) SGC feature propagation.

The hot path of bellaj09/SGC -- sgc_precompute (K hops of S.X, reference
utils.py:92-97) and the SGC linear classifier (models.py:7-18) -- on
hand-written HIP kernels behind a C ABI (include/sgc_amd.h,
libsgc_amd.so).  The reference's module surface is mirrored by
sgc_amd.utils / .models / .metrics / .args / .normalization, and re-exported
under the reference's own module names by dropin/.
"""
from .propagate import DeviceCSR, csr_of, linear, propagate, spmm  # noqa: F401

__all__ = ["DeviceCSR", "csr_of", "linear", "propagate", "spmm"]
