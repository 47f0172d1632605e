"""Time the classifier weight backward (sgc_linear_backward_f32) at the
Reddit-train shape: median per call over back-to-back calls (events), and
check it against fp64 torch.  Run once per library (SGC_AMD_LIB) for A/B.

    python scripts/bwd_ab.py [--rows 152410] [--features 602] [--classes 41]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd.classifier_bench import _median_ms  # noqa: E402
from sgc_amd.propagate import linear_backward  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=152410)
    ap.add_argument("--features", type=int, default=602)
    ap.add_argument("--classes", type=int, default=41)
    ap.add_argument("--kernel", type=int, default=0,
                    help="sgc_set_tuning('backward_kernel'): 0 auto, 1 fp32 slabs, 2 split-bf16 slabs, 3 split-bf16 column blocks")
    a = ap.parse_args()
    from sgc_amd import _lib
    _lib.check(_lib.load().sgc_set_tuning(b"backward_kernel", a.kernel), "set_tuning")
    g = torch.Generator().manual_seed(0)
    x = torch.randn(a.rows, a.features, generator=g)
    dy = torch.randn(a.rows, a.classes, generator=g) / a.rows
    xd, dyd = x.cuda(), dy.cuda()
    ms = _median_ms(lambda: linear_backward(xd, dyd), 20, inner=10)
    dW, db = linear_backward(xd, dyd)
    ref = dy.double().t() @ x.double()
    err = ((dW.cpu().double() - ref).abs().max() / ref.abs().max()).item()
    refb = dy.double().sum(0)
    errb = ((db.cpu().double() - refb).abs().max() / refb.abs().max()).item()
    name = _lib.load().sgc_linear_backward_kernel_name(a.rows, a.features, xd.stride(0),
                                                       a.classes,
                                                       _lib.ptr(xd)).decode()
    print(json.dumps({"lib": os.environ.get("SGC_AMD_LIB", "default"), "kernel": name,
                      "backward_ms": ms, "rel_err": err, "db_rel_err": errb}), flush=True)


if __name__ == "__main__":
    main()
