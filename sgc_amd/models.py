"""Drop-in for the reference's models.py: `SGC` and `get_model`.

SGC (reference models.py:7-18) is logistic regression over the propagated
features: an nn.Linear(nfeat, nclass) held as attribute `.W` (callers and
optimisers see the same parameters: .W.weight [nclass, nfeat], .W.bias).
On ROCm tensors the forward GEMM runs on the fp32 MFMA kernel
(sgc_linear_f32) and the weight backward (dW = dY^T X and db = sum dY, from
one read of X: sgc_linear_backward_f32) on the same MFMA tile -- what the
reference closures' .backward() needs (citation.py:47-49, reddit.py:55-58);
dX = dY W (only if the features require a gradient) is a torch op.  Adam
(citation.py:41) and LBFGS (reddit.py:52) work unchanged.  On CPU tensors (the reference's --no-cuda mode) the forward is the
reference's own nn.Linear arithmetic, so CPU runs reproduce its results bit
for bit.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .propagate import linear as _mfma_linear
from .propagate import linear_backward as _mfma_linear_backward
from .propagate import linear_xent as _fused_xent


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
        gw = gb = None
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_b:
            if weight.shape[0] <= 64:
                gw, gb = _mfma_linear_backward(x, grad_out, want_bias=want_b)
            else:  # wider than the fused kernel's 64 classes
                gw = grad_out.t() @ x
                gb = grad_out.sum(0) if want_b else None
            if not ctx.needs_input_grad[1]:
                gw = None
        return gx, gw, gb


class _LinearCrossEntropy(torch.autograd.Function):
    """loss = F.cross_entropy(x W^T + b, y) with dW, db from one fused pass
    (sgc_linear_xent_f32); the gradients are computed in forward and scaled
    by the incoming grad in backward."""

    @staticmethod
    def forward(ctx, x, weight, bias, labels):
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("fused SGC loss: no gradient w.r.t. the features")
        loss, dW, db = _fused_xent(x, weight, bias, labels)
        ctx.save_for_backward(dW, db if db is not None else dW.new_empty(0))
        ctx.has_bias = bias is not None
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        dW, db = ctx.saved_tensors
        return None, grad_loss * dW, (grad_loss * db if ctx.has_bias else None), None


def sgc_cross_entropy(model, features, labels):
    """F.cross_entropy(model(features), labels) for an SGC model, fused on the
    GPU: one launch chain computes the loss and the W/b gradients (the
    reference closure, citation.py:47-49 / reddit.py:55-58).  Works with Adam
    and LBFGS exactly like the unfused expression.  CPU tensors take the
    unfused expression itself."""
    if features.device.type == "cpu":
        return F.cross_entropy(model(features), labels)
    return _LinearCrossEntropy.apply(features, model.W.weight, model.W.bias, labels)


class SGC(nn.Module):
    """Logistic regression over S^K X (reference models.py:7-18)."""

    def __init__(self, nfeat, nclass):
        super().__init__()
        self.W = nn.Linear(nfeat, nclass)

    def forward(self, x):
        if x.device.type == "cpu":  # reference arithmetic (models.py:18)
            return self.W(x)
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
