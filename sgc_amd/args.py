"""Drop-in for the reference's args.py: get_citation_args() with the same
flags and defaults (reference args.py:4-40)."""
import argparse

import torch

_FLAGS = [
    # (flag, kwargs)
    ("--no-cuda", dict(action="store_true", default=False, help="Disables CUDA training.")),
    ("--seed", dict(type=int, default=42, help="Random seed.")),
    ("--epochs", dict(type=int, default=100, help="Number of epochs to train.")),
    ("--lr", dict(type=float, default=0.2, help="Initial learning rate.")),
    ("--weight_decay", dict(type=float, default=5e-6, help="Weight decay (L2 loss on parameters).")),
    ("--hidden", dict(type=int, default=0, help="Number of hidden units.")),
    ("--dropout", dict(type=float, default=0, help="Dropout rate (1 - keep probability).")),
    ("--dataset", dict(type=str, default="cora", help="Dataset to use.")),
    ("--model", dict(type=str, default="SGC", choices=["SGC", "GCN"], help="model to use.")),
    ("--feature", dict(type=str, default="mul", choices=["mul", "cat", "adj"], help="feature-type")),
    ("--normalization", dict(type=str, default="AugNormAdj", choices=["AugNormAdj"],
                             help="Normalization method for the adjacency matrix.")),
    ("--degree", dict(type=int, default=2, help="degree of the approximation.")),
    ("--per", dict(type=int, default=-1, help="Number of each nodes so as to balance.")),
    ("--experiment", dict(type=str, default="base-experiment", help="feature-type")),
    ("--tuned", dict(action="store_true", help="use tuned hyperparams")),
]


def get_citation_args(argv=None):
    parser = argparse.ArgumentParser()
    for flag, kw in _FLAGS:
        parser.add_argument(flag, **kw)
    args, _ = parser.parse_known_args(argv)
    args.cuda = not args.no_cuda and torch.cuda.is_available()
    return args
