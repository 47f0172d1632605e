"""LRU model of the light kernel's L2 reuse under row orderings (CPU only).

    gcc -O2 -o /tmp/lru_sim scripts/lru_sim.c && python scripts/locality_sim.py

For each ordering of scripts/locality_ab.py (the permuted CSR keeps every
row's nonzero sequence) and each row processing order (natural, or the
plan's length order), the fraction of X row-slice gathers that hit a per-XCD
LRU of 8192 slices (4 MB L2 / 512-B slice of 128 floats).  Beside it: the
share of nonzeros whose column is among the 8192 / 16384 most referenced
columns -- the order-free bound an LRU of that size approaches when the
graph has no community structure.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from sgc_amd import graphs  # noqa: E402
import locality_ab as L  # noqa: E402

SIM = os.environ.get("LRU_SIM", "/tmp/lru_sim")


def main():
    S = graphs.synthetic_graph("reddit", seed=0)
    freq = np.sort(np.bincount(S.col_idx, minlength=S.n))[::-1]
    cs = np.cumsum(freq) / S.nnz
    print(f"hot-column mass: top 8192 {cs[8191]:.3f}, top 16384 {cs[16383]:.3f}")
    td = tempfile.mkdtemp()
    for nm in ["identity", "rcm", "bfs", "degree"]:
        perm = L.ordering(S, nm)
        rp, ci, _ = L.permuted(S, perm)
        rp.astype(np.int32).tofile(os.path.join(td, "rp.bin"))
        ci.astype(np.int32).tofile(os.path.join(td, "ci.bin"))
        for proc, order in (("natural", np.arange(S.n)),
                            ("length", np.argsort(-np.diff(rp), kind="stable"))):
            order.astype(np.int32).tofile(os.path.join(td, "o.bin"))
            for cap in (8192, 16384):
                r = subprocess.run([SIM, str(S.n), str(S.nnz), os.path.join(td, "o.bin"),
                                    os.path.join(td, "rp.bin"), os.path.join(td, "ci.bin"),
                                    str(cap), "8", "8"], capture_output=True, text=True,
                                   check=True)
                print(f"{nm:9s} {proc:8s} cap {cap:6d}: {r.stdout.strip()}", flush=True)


if __name__ == "__main__":
    main()
