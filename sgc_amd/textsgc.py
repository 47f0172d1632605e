"""TextSGC's one-hop feature precompute on the MI355X engine (SURVEY.md 8(f)
row 4) -- drop-in for sgc_precompute in the reference's
downstream/TextSGC/utils.py:131-152 (same signature, same return).

The TextSGC app (train.py:103-106) passes the normalised doc/word adjacency
`adj` and `features` = adj as a dense matrix, with degree = 1: for each
split, F = (S . features[:, idx])^T -- one SpMM whose right-hand side is the
split's columns of S -- then columns with zero range over the training rows
are dropped and every split is min/range-scaled with the training statistics.
The SpMM runs on the HIP kernel (bit-exact with torch.spmm's CPU kernel); the
transpose, min/max, filter and scaling are elementwise torch ops on the
device.  As in the reference, train stays on the device and val/test come
back to the host.
"""
from time import perf_counter

import numpy as np
import torch

from .propagate import csr_of, spmm


def sparse_to_torch_sparse(sparse_mx, device="cuda"):
    """scipy -> torch sparse COO fp32 (reference TextSGC utils.py:103-118)."""
    coo = sparse_mx.tocoo().astype(np.float32)
    indices = torch.from_numpy(np.vstack((coo.row, coo.col)).astype(np.int64))
    return torch.sparse_coo_tensor(indices, torch.from_numpy(coo.data),
                                   torch.Size(coo.shape)).to(device)


def sparse_to_torch_dense(sparse, device="cuda"):
    """(reference TextSGC utils.py:120-123)"""
    return torch.from_numpy(np.asarray(sparse.todense()).astype(np.float32)).to(device=device)


def sgc_precompute(adj, features, degree, index_dict):
    """(feat_dict, seconds) exactly as the reference's TextSGC sgc_precompute;
    adj must be on the ROCm device (the reference moves it there too)."""
    assert degree == 1, "Only supporting degree 2 now"  # the reference's message
    dev = adj.device
    if dev.type != "cuda":
        raise RuntimeError("sgc_amd.textsgc: adj must be on the ROCm device (no CPU fallback)")
    torch.cuda.synchronize(dev)
    start = perf_counter()
    csr = csr_of(adj)

    def hop(idx):
        X = features[:, idx].to(dev, non_blocking=True).contiguous()
        return spmm(csr, X).t()

    feat_dict = {}
    train_feats = hop(index_dict["train"])
    train_feats_max, _ = train_feats.max(dim=0, keepdim=True)
    train_feats_min, _ = train_feats.min(dim=0, keepdim=True)
    train_feats_range = train_feats_max - train_feats_min
    useful = train_feats_range.squeeze().gt(0).nonzero().squeeze()
    train_feats = train_feats[:, useful]
    train_feats_range = train_feats_range[:, useful]
    train_feats_min = train_feats_min[:, useful]
    feat_dict["train"] = (train_feats - train_feats_min) / train_feats_range
    for phase in ["test", "val"]:
        feats = hop(index_dict[phase])[:, useful]
        feat_dict[phase] = ((feats - train_feats_min) / train_feats_range).cpu()
    torch.cuda.synchronize(dev)
    return feat_dict, perf_counter() - start
