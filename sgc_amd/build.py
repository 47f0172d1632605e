"""Build libsgc_amd.so (gfx950) in-tree with hipcc.

The shared library is the product's native core: HIP kernels for gfx950 plus
the C ABI in include/sgc_amd.h.  It is built in-tree so it travels with the
repo snapshot to the GPU box (see .gitignore: *.so stays out of history).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libsgc_amd.so")
SOURCES = ["capi.hip", "spmm.hip", "ingest.hip", "linear.hip", "normalize.hip", "xent.hip",
           "subgraph.hip", "cpu.hip"]


def _headers():
    """Every header a source may include (csrc/*.h and the public ABI)."""
    import glob
    return sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include",
                                                                        "sgc_amd.h")]
ARCH = os.environ.get("SGC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    # IEEE fp32: no FTZ, no contraction beyond the explicit fmaf chains
    "-fno-gpu-flush-denormals-to-zero",
    "-ffp-contract=off",
    "-fno-fast-math",
    "-Wall",
    "-Wno-unused-function",
]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES] + _headers()
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True, out=None, defines=()):
    """Compile the library; `out`/`defines` build tuning variants elsewhere."""
    lib = out or LIB
    if not force and out is None and not _stale():
        return LIB
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    tmp = lib + ".tmp"
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in defines], "-I", os.path.join(ROOT, "include"),
           "-I", CSRC, *srcs, "-o", tmp]
    if verbose:
        print("[sgc_amd] " + " ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv)
