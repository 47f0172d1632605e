"""Drop-in for the reference's models.py: `SGC` and `get_model`.

SGC (reference models.py:7-18) is logistic regression over the propagated
features: an nn.Linear(nfeat, nclass) held as attribute `.W` (callers and
optimisers see the same parameters: .W.weight [nclass, nfeat], .W.bias).
The forward GEMM runs on the fp32 MFMA kernel (sgc_linear_f32); the backward
(dW = dY^T X, db = sum dY, dX = dY W) is three small torch ops, so Adam
(citation.py:41) and LBFGS (reddit.py:52) work unchanged.
"""
import torch
import torch.nn as nn

from .propagate import linear as _mfma_linear


class _LinearMFMA(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return _mfma_linear(x, weight, bias)

    @staticmethod
    def backward(ctx, grad_out):
        x, weight = ctx.saved_tensors
        gx = grad_out @ weight if ctx.needs_input_grad[0] else None
        gw = grad_out.t() @ x if ctx.needs_input_grad[1] else None
        gb = grad_out.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw, gb


class SGC(nn.Module):
    """Logistic regression over S^K X (reference models.py:7-18)."""

    def __init__(self, nfeat, nclass):
        super().__init__()
        self.W = nn.Linear(nfeat, nclass)

    def forward(self, x):
        return _LinearMFMA.apply(x, self.W.weight, self.W.bias)


def get_model(model_opt, nfeat, nclass, nhid=0, dropout=0, cuda=True):
    """(reference models.py:59-72).  Only "SGC" is built: the reference's GCN
    is broken there (GraphConvolution.forward returns None, models.py:36-38)
    and out of this engine's scope; any other name raises
    NotImplementedError like the reference."""
    if model_opt == "SGC":
        model = SGC(nfeat=nfeat, nclass=nclass)
    elif model_opt == "GCN":
        raise NotImplementedError("model:GCN is not provided by sgc_amd (broken in the reference, "
                                  "models.py:36-38)")
    else:
        raise NotImplementedError("model:{} is not implemented!".format(model_opt))
    if cuda:
        model.cuda()
    return model
