"""Drop-in for the reference's utils.py: same names, arguments and return
values, with the propagation running on the MI355X engine.

    from utils import load_citation, sgc_precompute, set_seed     # citation.py:7
    from utils import load_reddit_data, sgc_precompute, set_seed  # reddit.py:7

Hot path: sgc_precompute (reference utils.py:92-97).  Differences, all on the
timing side: the clock is read after a device synchronise (the reference's
GPU timer is not synchronised, utils.py:93,96), and the first call on a new
adjacency includes its COO->CSR ingest (cached afterwards; the ingest time is
also kept on the CSR as `ingest_seconds`).
"""
import os
import pickle as pkl
import sys
from time import perf_counter

import numpy as np
import scipy.sparse as sp
import torch

from . import multigpu
from .normalization import aug_normalize_on_device, fetch_normalization, row_normalize
from .propagate import check_propagation_inputs, csr_of, propagate, to_torch_coo, warmup

# under torchrun: this process's `.cuda()` is its own GPU (cuda:LOCAL_RANK),
# so an unchanged reddit.py / citation.py spreads over the node's GPUs
multigpu.bind_local_device()


def parse_index_file(filename):
    """One integer per line (reference utils.py:10-15)."""
    with open(filename) as f:
        return [int(line.strip()) for line in f]


def preprocess_citation(adj, features, normalization="FirstOrderGCN"):
    """(reference utils.py:17-21)"""
    return fetch_normalization(normalization)(adj), row_normalize(features)


def sparse_mx_to_torch_sparse_tensor(sparse_mx):
    """scipy -> torch sparse COO fp32, int64 [2,nnz] indices in .tocoo() order
    (reference utils.py:23-30).  Not coalesced, like the reference's."""
    coo = sparse_mx.tocoo().astype(np.float32)
    indices = torch.from_numpy(np.stack([coo.row, coo.col]).astype(np.int64))
    values = torch.from_numpy(coo.data)
    return torch.sparse_coo_tensor(indices, values, torch.Size(coo.shape))


def _normalized_adj(adj, normalization, cuda):
    """The loaders' adjacency: AugNorm on the GPU when it applies (canonical A,
    'AugNormAdj', cuda) -- bit-identical to the reference's host scipy path and
    ~1000x faster at Reddit shape -- else the reference's host path."""
    a = sp.csr_matrix(adj)
    if cuda and normalization == "AugNormAdj" and a.has_canonical_format:
        return to_torch_coo(aug_normalize_on_device(a, "cuda"))
    t = sparse_mx_to_torch_sparse_tensor(fetch_normalization(normalization)(adj)).float()
    return t.cuda() if cuda else t


def _reddit_adjs(adj, train_index, normalization, cuda):
    """(S, S_train) for load_reddit_data (reference utils.py:116-124): the
    train sub-graph is sliced from A + A^T BEFORE normalisation.  On the GPU
    (canonical A, 'AugNormAdj', distinct train ids) A is uploaded once and both
    the slice (sgc_subgraph_*) and both normalisations run on the device --
    bit-identical to the reference's scipy path; otherwise the host path."""
    a = sp.csr_matrix(adj)
    idx = np.asarray(train_index, dtype=np.int64)
    if (cuda and normalization == "AugNormAdj" and a.has_canonical_format
            and np.unique(idx).size == idx.size):
        from .normalization import aug_normalize_device_arrays, device_csr64, subgraph_on_device
        rp, ci, va, n = device_csr64(a, "cuda")
        full = to_torch_coo(aug_normalize_device_arrays(rp, ci, va, n))
        sub = to_torch_coo(aug_normalize_device_arrays(*subgraph_on_device(rp, ci, va, n, idx)))
        return full, sub
    return (_normalized_adj(adj, normalization, cuda),
            _normalized_adj(adj[idx, :][:, idx], normalization, cuda))


def sgc_precompute(features, adj, degree):
    """X_K = S^K X; returns (features_K, seconds) like utils.py:92-97.

    ROCm tensors run on the HIP kernels, CPU tensors on the library's host
    twin (the reference's --no-cuda mode); mixed devices raise RuntimeError.
    degree <= 0 returns the input tensor object itself (the reference's loop
    body never runs).  The result is bit-identical to the reference's
    torch.spmm chain on CPU for the same inputs, on either device -- and on
    any number of GPUs: under torchrun (or an initialised process group of
    world > 1) the hops run partitioned over the ranks and every rank gets
    the whole X_K; with SGC_AMD_DEVICES one process drives several GPUs
    (sgc_amd.multigpu)."""
    if degree <= 0:
        t = perf_counter()
        return features, perf_counter() - t
    dev = features.device
    if dev.type == "cuda" and not torch.cuda.current_stream(dev).query():
        _synchronize(dev)  # earlier work on the caller's stream stays out of the time
    t = perf_counter()
    csr = csr_of(adj)
    out = _propagate_on_node(csr, features, degree)
    if dev.type == "cuda":
        # every path joins its work (side streams, RCCL, other devices) back
        # to the caller's stream, so that stream's completion is X_K's
        torch.cuda.current_stream(dev).synchronize()
    return out, perf_counter() - t


def _synchronize(dev):
    """torch.cuda.synchronize(dev) without its device switch when dev is the
    current device (the switch costs ~1 us a call: Pubmed-shape calls are
    ~0.1 ms)."""
    if dev.index is None or dev.index == torch.cuda.current_device():
        torch.cuda.synchronize()
    else:
        torch.cuda.synchronize(dev)


def _propagate_on_node(csr, X, K):
    """One GPU, the process group's GPUs, or this process's device set."""
    group = multigpu.process_group(X.device)
    if group is not None:
        X = check_propagation_inputs(csr, X)
        return multigpu.precompute_group(csr, X, K, group)
    if X.device.type == "cuda":
        devices = multigpu.devices_from_env(X.device.index)
        if devices:
            X = check_propagation_inputs(csr, X)
            return multigpu.precompute_devices(csr, X, K, devices)
    return propagate(csr, X, K)


def set_seed(seed, cuda):
    """(reference utils.py:99-102)"""
    np.random.seed(seed)
    torch.manual_seed(seed)
    if cuda:
        torch.cuda.manual_seed(seed)


def load_citation(dataset_str="cora", normalization="AugNormAdj", cuda=True):
    """Planetoid loader with the reference's semantics (utils.py:32-90).

    Reads data/ind.<dataset>.{x,y,tx,ty,allx,ally,graph} (pickles: the user's
    own dataset files) and data/ind.<dataset>.test.index from the working
    directory, fixes Citeseer's isolated test nodes, symmetrises A by
    elementwise max, applies the normalisation and row-normalises features.
    Returns (adj, features, labels, idx_train, idx_val, idx_test)."""
    import networkx as nx
    objs = {}
    for name in ("x", "y", "tx", "ty", "allx", "ally", "graph"):
        with open(f"data/ind.{dataset_str.lower()}.{name}", "rb") as f:
            objs[name] = pkl.load(f, encoding="latin1") if sys.version_info > (3, 0) else pkl.load(f)
    x, y, tx, ty, allx, ally, graph = (objs[k] for k in ("x", "y", "tx", "ty", "allx", "ally", "graph"))
    test_idx_reorder = parse_index_file(f"data/ind.{dataset_str}.test.index")
    test_idx_range = np.sort(test_idx_reorder)

    if dataset_str == "citeseer":
        # isolated test nodes: zero rows at their positions
        lo, hi = min(test_idx_reorder), max(test_idx_reorder)
        tx_full = sp.lil_matrix((hi - lo + 1, x.shape[1]))
        tx_full[test_idx_range - lo, :] = tx
        tx = tx_full
        ty_full = np.zeros((hi - lo + 1, y.shape[1]))
        ty_full[test_idx_range - lo, :] = ty
        ty = ty_full

    features = sp.vstack((allx, tx)).tolil()
    features[test_idx_reorder, :] = features[test_idx_range, :]
    adj = nx.adjacency_matrix(nx.from_dict_of_lists(graph))
    upper = adj.T > adj
    adj = adj + adj.T.multiply(upper) - adj.multiply(upper)
    labels = np.vstack((ally, ty))
    labels[test_idx_reorder, :] = labels[test_idx_range, :]

    idx_test = test_idx_range.tolist()
    idx_train = range(len(y))
    idx_val = range(len(y), len(y) + 500)

    features = row_normalize(features)
    adj = _normalized_adj(adj, normalization, cuda)

    features = torch.FloatTensor(np.array(features.todense())).float()
    labels = torch.LongTensor(labels).max(dim=1)[1]
    idx_train, idx_val, idx_test = (torch.LongTensor(i) for i in (idx_train, idx_val, idx_test))
    if cuda:
        features, labels = features.cuda(), labels.cuda()
        idx_train, idx_val, idx_test = idx_train.cuda(), idx_val.cuda(), idx_test.cuda()
        warmup()  # the engine's code objects load here, not in the timed precompute
    return adj, features, labels, idx_train, idx_val, idx_test


def loadRedditFromNPZ(dataset_dir):  # noqa: N802  (reference name)
    """(reference utils.py:104-108) -- npz only, no pickles."""
    adj = sp.load_npz(dataset_dir + "reddit_adj.npz")
    data = np.load(dataset_dir + "reddit.npz")
    return (adj, data["feats"], data["y_train"], data["y_val"], data["y_test"],
            data["train_index"], data["val_index"], data["test_index"])


def load_reddit_data(data_path="data/", normalization="AugNormAdj", cuda=True):
    """(reference utils.py:110-131), quirks kept: reddit.py:38 passes the
    normalisation name positionally into data_path, so a data_path that is not
    an existing directory falls back to "data/" (the reference always reads
    "data/"); `cuda` defaults to True.  adj = A + A^T; the train subgraph is
    sliced before normalisation; features standardised per column."""
    if not (isinstance(data_path, str) and os.path.isdir(data_path)):
        data_path = "data/"
    if not data_path.endswith("/"):
        data_path += "/"
    adj, features, y_train, y_val, y_test, train_index, val_index, test_index = \
        loadRedditFromNPZ(data_path)
    labels = np.zeros(adj.shape[0])
    labels[train_index] = y_train
    labels[val_index] = y_val
    labels[test_index] = y_test
    adj = adj + adj.T
    features = torch.FloatTensor(np.array(features))
    features = (features - features.mean(dim=0)) / features.std(dim=0)
    adj, train_adj = _reddit_adjs(adj, train_index, normalization, cuda)
    labels = torch.LongTensor(labels)
    if cuda:
        features, labels = features.cuda(), labels.cuda()
        warmup()  # the engine's code objects load here, not in the timed precompute
    return adj, train_adj, features, labels, train_index, val_index, test_index
