"""ctypes binding of libsgc_amd.so (C ABI: include/sgc_amd.h).

The product path always runs the HIP kernels: if the library is missing or
cannot be loaded, every call raises -- there is no CPU or torch fallback.
torch is imported first so the library's libamdhip64.so.7 dependency binds to
the HIP runtime torch already loaded (one runtime per process).
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see above)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SGC_AMD_LIB", os.path.join(_HERE, "libsgc_amd.so"))

_i64, _i32, _u32 = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32
_p, _sz = ctypes.c_void_p, ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/sgc_amd.h one for one.
SIGNATURES = {
    "sgc_abi_version": (ctypes.c_int, []),
    "sgc_last_error": (ctypes.c_char_p, []),
    "sgc_set_tuning": (ctypes.c_int, [ctypes.c_char_p, _i64]),
    "sgc_get_tuning": (_i64, [ctypes.c_char_p]),
    "sgc_coo_to_csr_workspace": (ctypes.c_int, [_i64, _i64, ctypes.POINTER(_sz)]),
    "sgc_coo_to_csr": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _i64, _p, _p, _p, _p, _sz,
                                      ctypes.POINTER(_u32), _p]),
    "sgc_csr64_to_csr": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _i64, _p, _p, _p,
                                        ctypes.POINTER(_u32), _p]),
    "sgc_augnorm_workspace": (_i64, [_i64]),
    "sgc_augnorm_count": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _p, _p, _p, _i64,
                                         ctypes.POINTER(_i64), ctypes.POINTER(_u32), _p]),
    "sgc_augnorm_fill": (ctypes.c_int, [_p, _p, _p, _i64, _p, _p, _p, _p, _p, _i64,
                                        ctypes.POINTER(_i64), _p]),
    "sgc_csr_to_coo64": (ctypes.c_int, [_p, _p, _i64, _p, _p, _p]),
    "sgc_subgraph_workspace": (_i64, [_i64, _i64, _i64]),
    "sgc_subgraph_count": (ctypes.c_int, [_p, _p, _i64, _i64, _p, _i64, _p, _p, _i64,
                                          ctypes.POINTER(_i64), ctypes.POINTER(_u32), _p]),
    "sgc_subgraph_fill": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _p, _i64, _p, _p, _p, _p, _i64,
                                         _p]),
    "sgc_plan_capacity": (_i64, [_i64]),
    "sgc_plan_build": (ctypes.c_int, [_p, _i64, _i64, _i32, _i32, _p, _i64, ctypes.POINTER(_i64),
                                      ctypes.POINTER(_i64), _p]),
    "sgc_plan_light_order": (ctypes.c_int, [_p, _i64, _i64, _i32, _p, ctypes.POINTER(_i64), _p]),
    "sgc_spmm_csr_f32": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64,
                                        _p, _i64, _i64, _i32, _p]),
    "sgc_spmm_csr_f32_ex": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64,
                                           _p, _i64, _i64, _i32, _u32, _p]),
    "sgc_propagate_workspace": (_i64, [_i64, _i64, _i64, _i32]),
    "sgc_propagate_f32": (ctypes.c_int, [_p, _p, _p, _i64, _p, _i64, _p, _i64, _i64, _i32,
                                         _p, _i64, _i64, _i32, _p, _i64, _p]),
    "sgc_propagate_groups_f32": (ctypes.c_int, [_i32, _p, _p, _p, _i64, _p, _i64, _p, _i64, _i64,
                                                 _i32, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "sgc_pad_rows_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _i64, _i64, _p]),
    "sgc_copy_blocks_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _i32, _p, _p]),
    "sgc_ipc_get_handle": (ctypes.c_int, [_p, _p]),
    "sgc_ipc_open": (ctypes.c_int, [_p, ctypes.POINTER(_p), ctypes.POINTER(_p)]),
    "sgc_ipc_close": (ctypes.c_int, [_p]),
    "sgc_signal_flag_i32": (ctypes.c_int, [_p, _i32, _p]),
    "sgc_wait_flags_i32": (ctypes.c_int, [_i32, _p, _i32, _p, _i64, _p]),
    "sgc_pull_blocks_f32": (ctypes.c_int, [_i32, _p, _p, _i64, _p]),
    "sgc_aligned_ld": (_i64, [_i64]),
    "sgc_launch_list_create": (ctypes.c_int, [ctypes.POINTER(_i64)]),
    "sgc_launch_list_add_spmm": (ctypes.c_int, [_i64, _p, _p, _p, _i64, _i64, _p, _i64, _p, _i64,
                                                _i64, _p, _i64, _i64, _i32, _u32, _i32, _i32]),
    "sgc_launch_list_add_pad_rows": (ctypes.c_int, [_i64, _p, _i64, _p, _i64, _i64, _i64, _i32,
                                                    _i32]),
    "sgc_launch_list_run": (ctypes.c_int, [_i64, _p, _p, _p]),
    "sgc_launch_list_destroy": (ctypes.c_int, [_i64]),
    "sgc_linear_f32": (ctypes.c_int, [_p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "sgc_linear_kernel_name": (ctypes.c_char_p, [_i64, _i64, _i64, _i64, _p]),
    "sgc_linear_backward_kernel_name": (ctypes.c_char_p, [_i64, _i64, _i64, _i64, _p]),
    "sgc_cross_entropy_workspace": (_i64, [_i64, _i64]),
    "sgc_cross_entropy_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _i64, _i64, _p, _p, _p, _p, _i64,
                                             _p]),
    "sgc_cross_entropy_backward_f32": (ctypes.c_int, [_p, _i64, _p, _p, _p, _p, _i64, _i64, _i64,
                                                      _p, _i64, _p]),
    "sgc_linear_xent_workspace": (_i64, [_i64, _i64, _i64]),
    "sgc_linear_xent_f32": (ctypes.c_int, [_p, _i64, _p, _p, _p, _i64, _i64, _i64, _p, _p, _p,
                                           _p, _i64, _p, _i64, _p]),
    "sgc_timing_enable": (ctypes.c_int, [ctypes.c_int]),
    "sgc_timing_collect": (ctypes.c_int, [_p, _p, _i64, ctypes.POINTER(_i64)]),
    "sgc_timing_collect_ex": (ctypes.c_int, [_p, _p, _p, _p, _i64, ctypes.POINTER(_i64)]),
    "sgc_coo_to_csr_cpu": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _i64, _p, _p, _p,
                                          ctypes.POINTER(_u32)]),
    "sgc_spmm_csr_f32_cpu": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64,
                                            _i32]),
    "sgc_spmm_csr_f32_cpu_ex": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _p, _i64, _p, _i64, _i64,
                                               ctypes.c_uint32, _i32]),
    "sgc_propagate_cpu_workspace": (_i64, [_i64, _i64, _i32]),
    "sgc_propagate_f32_cpu": (ctypes.c_int, [_p, _p, _p, _i64, _p, _i64, _p, _i64, _i64, _i32,
                                             _p, _i64, _i32]),
    "sgc_colsplit_workspace": (_i64, [_i64, _i32]),
    "sgc_csr_colsplit": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _i32, _p, _p, _p, _p, _p, _i64,
                                        _p]),
    "sgc_plan_sorted_workspace": (_i64, [_i64]),
    "sgc_plan_sorted": (ctypes.c_int, [_p, _i64, _i64, _i32, _i32, _p, _p, _i64, _p, _p]),
    "sgc_mgpu_init": (ctypes.c_int, [ctypes.c_int, _p]),
    "sgc_mgpu_attach": (ctypes.c_int, [_p, _p, _p, _i64, _i64, _p, ctypes.POINTER(_i64)]),
    "sgc_mgpu_propagate": (ctypes.c_int, [_i64, _p, _i64, _p, _i64, _i64, _i32, _p]),
    "sgc_mgpu_detach": (ctypes.c_int, [_i64]),
    "sgc_mgpu_finalize": (ctypes.c_int, []),
    "sgc_warmup": (ctypes.c_int, [_u32, _p]),
    "sgc_linear_backward_workspace": (_i64, [_i64, _i64, _i64]),
    "sgc_linear_backward_f32": (ctypes.c_int, [_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _p, _p,
                                               _i64, _p]),
}

ABI_VERSION = 1
_lib = None


class SGCError(RuntimeError):
    pass


def load_path(path):
    """Load and type one build of the library (tuning scripts load several)."""
    if not os.path.exists(path):
        raise SGCError(
            f"sgc_amd: native library {path} not found; build it with "
            "`python -m sgc_amd.build` (hipcc --offload-arch=gfx950). "
            "There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.sgc_abi_version() != ABI_VERSION:
        raise SGCError(f"sgc_amd: ABI mismatch ({lib.sgc_abi_version()} != {ABI_VERSION})")
    return lib


def load():
    """Load and type the product library (once).  Raises if it is absent."""
    global _lib
    if _lib is None:
        _lib = load_path(LIB_PATH)
    return _lib


def check(rc, what):
    if rc != 0:
        msg = load().sgc_last_error().decode(errors="replace")
        raise SGCError(f"sgc_amd: {what} failed (code {rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
