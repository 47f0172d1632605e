"""Time the logits cross-entropy kernels (sgc_cross_entropy_f32 forward, and
_backward_f32) at the Reddit-train shape through the drop-in route the
reference closures take, F.cross_entropy on SGC's logits: median ms per call
over back-to-back calls (events), checked against fp64 torch.  Run once per
library (SGC_AMD_LIB) for A/B.

    python scripts/ce_ab.py [--rows 152410] [--classes 41]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd.classifier_bench import _median_ms  # noqa: E402
from sgc_amd.models import SGCLogits  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=152410)
    ap.add_argument("--classes", type=int, default=41)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    y = torch.randn(a.rows, a.classes, generator=g) * 4
    t = torch.randint(0, a.classes, (a.rows,), generator=g)
    yd, td = y.cuda(), t.cuda()
    logits = yd.as_subclass(SGCLogits)
    fwd = _median_ms(lambda: F.cross_entropy(logits, td), 20, inner=10)
    leaf = yd.clone().requires_grad_(True)

    def both():
        loss = F.cross_entropy(leaf.as_subclass(SGCLogits), td)
        loss.backward()
        leaf.grad = None
    fb = _median_ms(both, 20, inner=10)
    leaf.grad = None
    loss = F.cross_entropy(leaf.as_subclass(SGCLogits), td)
    loss.backward()
    yr = y.double().requires_grad_(True)
    ref = F.cross_entropy(yr, t)
    ref.backward()
    print(json.dumps({"lib": os.environ.get("SGC_AMD_LIB", "default"), "forward_ms": fwd,
                      "fwd_bwd_ms": fb, "loss_err": abs(loss.item() - ref.item()),
                      "grad_err": (leaf.grad.cpu().double() - yr.grad).abs().max().item()}),
          flush=True)


if __name__ == "__main__":
    main()
