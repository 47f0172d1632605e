"""Citation-network driver on the MI355X engine -- counterpart of the
reference's citation.py (same flags via get_citation_args, same output
lines), reading Planetoid files from ./data like the reference.

    python drivers/citation.py --dataset cora [--tuned] [--degree 2] [--epochs 100]

Flow (reference citation.py:14-70): seed -> load_citation -> SGC model
(created before the precompute, so the RNG draws for W match) ->
sgc_precompute on the GPU -> Adam over the training rows -> accuracy.
--tuned uses the tuned weight decays of the reference's SGC-tuning/ results
(values recorded in SURVEY.md section 2, row 11; the pickled files are not
read).
"""
import os
import sys
from time import perf_counter

import torch
import torch.nn.functional as F
import torch.optim as optim

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sgc_amd.args import get_citation_args  # noqa: E402
from sgc_amd.metrics import accuracy  # noqa: E402
from sgc_amd.models import get_model  # noqa: E402
from sgc_amd.utils import load_citation, set_seed, sgc_precompute  # noqa: E402

TUNED_WEIGHT_DECAY = {"cora": 1.3027e-05, "citeseer": 2.3546e-05, "pubmed": 7.4039e-05}


def train_regression(model, train_features, train_labels, val_features, val_labels,
                     epochs, weight_decay, lr, dropout):
    optimizer = optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)
    t = perf_counter()
    for _ in range(epochs):
        model.train()
        optimizer.zero_grad()
        loss = F.cross_entropy(model(train_features), train_labels)
        loss.backward()
        optimizer.step()
    train_time = perf_counter() - t
    with torch.no_grad():
        model.eval()
        acc_val = accuracy(model(val_features), val_labels)
    return model, acc_val, train_time


def test_regression(model, test_features, test_labels):
    model.eval()
    return accuracy(model(test_features), test_labels)


def main(argv=None):
    args = get_citation_args(argv)
    if args.tuned:
        if args.model != "SGC":
            raise NotImplementedError("tuned hyper-parameters exist for SGC only")
        args.weight_decay = TUNED_WEIGHT_DECAY[args.dataset]
        print("using tuned weight decay: {}".format(args.weight_decay))
    set_seed(args.seed, args.cuda)
    adj, features, labels, idx_train, idx_val, idx_test = load_citation(
        args.dataset, args.normalization, args.cuda)
    model = get_model(args.model, features.size(1), labels.max().item() + 1, args.hidden,
                      args.dropout, args.cuda)
    features, precompute_time = sgc_precompute(features, adj, args.degree)
    print("{:.4f}s".format(precompute_time))
    model, acc_val, train_time = train_regression(
        model, features[idx_train], labels[idx_train], features[idx_val], labels[idx_val],
        args.epochs, args.weight_decay, args.lr, args.dropout)
    acc_test = test_regression(model, features[idx_test], labels[idx_test])
    print("Validation Accuracy: {:.4f} Test Accuracy: {:.4f}".format(acc_val, acc_test))
    print("Pre-compute time: {:.4f}s, train time: {:.4f}s, total: {:.4f}s".format(
        precompute_time, train_time, precompute_time + train_time))
    return float(acc_val), float(acc_test)


if __name__ == "__main__":
    main()
