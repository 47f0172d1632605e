"""Write the Reddit-shape S's column ids in CSR order (int32) for gather_rate.

    python scripts/micro/gather_cols.py OUT.bin [--shape reddit]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from sgc_amd import graphs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--shape", default="reddit")
a = ap.parse_args()
S = graphs.synthetic_graph(a.shape, seed=0)
S.col_idx.astype("int32").tofile(a.out)
print(f"{a.out}: {S.nnz} column ids, n = {S.n}")
