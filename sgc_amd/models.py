"""Drop-in for the reference's models.py: `SGC` and `get_model`.

SGC (reference models.py:7-18) is logistic regression over the propagated
features: an nn.Linear(nfeat, nclass) held as attribute `.W` (callers and
optimisers see the same parameters: .W.weight [nclass, nfeat], .W.bias).
On ROCm tensors the forward GEMM runs on the fp32 MFMA kernel
(sgc_linear_f32) and the weight backward (dW = dY^T X and db = sum dY, from
one read of X: sgc_linear_backward_f32) on the same MFMA tile -- what the
reference closures' .backward() needs (citation.py:47-49, reddit.py:55-58);
dX = dY W (only if the features require a gradient) is a torch op.  Adam
(citation.py:41) and LBFGS (reddit.py:52) work unchanged.  The ROCm output is
an SGCLogits tensor: the closures' unchanged F.cross_entropy(output, labels)
runs on the HIP cross-entropy kernels (sgc_cross_entropy_f32, one pass for
the loss, one for the gradient) rather than torch's nll reduction.  On CPU
tensors (the reference's --no-cuda mode) the forward is the
reference's own nn.Linear arithmetic, so CPU runs reproduce its results bit
for bit.

Non-finite inputs: the GPU forward's split-bf16 kernel (the default for
M >= 4096 where W fits LDS) needs finite features and weights within bf16's
range (|x| <= 3.39e38): an infinite (or larger) x or w inside the K range
gives NaN in its row's logits where torch gives +-inf (tests pin it:
test_linear_split_nonfinite_inside_k).  SGC's propagated features are finite;
a caller that needs torch's non-finite semantics selects the fp32 kernel with
sgc_set_tuning("linear_kernel", 2).
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


class _LogitsCrossEntropy(torch.autograd.Function):
    """F.cross_entropy(logits, labels) (mean, ignore_index) on the HIP kernels
    (sgc_cross_entropy_f32 / _backward_f32): the loss and the per-row
    log-sum-exp in one pass, the logits' gradient in one more -- scaled by
    the incoming gradient on the device, no host synchronisation."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        from . import _lib
        lib = _lib.load()
        M, C = logits.shape
        dev = logits.device
        _check_labels(labels, C, ignore_index)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        inv = torch.empty(1, dtype=torch.float32, device=dev)
        lse = torch.empty(M, dtype=torch.float32, device=dev)
        ws_bytes = lib.sgc_cross_entropy_workspace(M, C)
        ws = torch.empty(max(1, ws_bytes), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            _lib.check(lib.sgc_cross_entropy_f32(_lib.ptr(logits), logits.stride(0), _lib.ptr(labels),
                                                 M, C, int(ignore_index), _lib.ptr(loss), _lib.ptr(inv),
                                                 _lib.ptr(lse), _lib.ptr(ws), ws_bytes,
                                                 _lib.stream_handle(dev)), "cross_entropy_f32")
        ctx.save_for_backward(logits, labels, lse, inv)
        ctx.ignore_index = int(ignore_index)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable  # (a double backward raises, never silently zero)
    def backward(ctx, grad_loss):
        from . import _lib
        logits, labels, lse, inv = ctx.saved_tensors
        M, C = logits.shape
        dY = torch.empty((M, C), dtype=torch.float32, device=logits.device)
        g = grad_loss.detach().to(torch.float32).contiguous()
        with torch.cuda.device(logits.device):
            _lib.check(_lib.load().sgc_cross_entropy_backward_f32(
                _lib.ptr(logits), logits.stride(0), _lib.ptr(labels), _lib.ptr(lse), _lib.ptr(inv),
                _lib.ptr(g), M, C, ctx.ignore_index, _lib.ptr(dY), dY.stride(0),
                _lib.stream_handle(logits.device)), "cross_entropy_backward_f32")
        return dY, None, None


_checked_labels = {}


def _check_labels(labels, C, ignore_index):
    """Raise, as torch does ("Target ... is out of bounds"), for a label
    outside [0, C) that is not ignore_index -- the HIP loss would otherwise
    return NaN and poison the optimiser's weights.  One check (and one host
    synchronisation) per labels tensor and version: the reference closures
    pass the same labels tensor on every call (citation.py:46-49,
    reddit.py:55-58), so LBFGS's 20-odd closures per step pay it once."""
    key = (labels.data_ptr(), labels._version, labels.shape[0], int(C), int(ignore_index))
    if key in _checked_labels:
        return
    bad = ((labels < 0) | (labels >= C)) & (labels != ignore_index)
    if bool(bad.any()):
        y = int(labels[bad][0])
        raise IndexError(f"Target {y} is out of bounds (classes: {C}, ignore_index: "
                         f"{ignore_index})")
    if len(_checked_labels) > 64:
        _checked_labels.clear()
    _checked_labels[key] = True


def _cross_entropy_args(args, kwargs):
    """(logits, labels, ignore_index) when F.cross_entropy(*args, **kwargs) is
    the plain form the HIP kernels compute (mean reduction, no class weights,
    no label smoothing, int64 class-index labels, C <= 64), else None."""
    names = ("input", "target", "weight", "size_average", "ignore_index", "reduce", "reduction",
             "label_smoothing")
    bound = dict(zip(names, args))
    for k, v in kwargs.items():
        if k in bound or k not in names:
            return None
        bound[k] = v
    x, y = bound.get("input"), bound.get("target")
    if (bound.get("weight") is not None or bound.get("size_average") is not None or
            bound.get("reduce") is not None or bound.get("reduction", "mean") != "mean" or
            bound.get("label_smoothing", 0.0) != 0.0):
        return None
    if not (isinstance(x, torch.Tensor) and isinstance(y, torch.Tensor)):
        return None
    if (x.dim() != 2 or x.dtype != torch.float32 or x.device.type != "cuda" or
            not 0 < x.shape[1] <= 64 or x.shape[0] == 0 or x.stride(1) != 1 or
            x.stride(0) < x.shape[1] or
            y.dim() != 1 or y.dtype != torch.int64 or y.device != x.device or
            y.shape[0] != x.shape[0]):
        return None
    return x, y.contiguous(), int(bound.get("ignore_index", -100))


class SGCLogits(torch.Tensor):
    """The ROCm classifier's output (SGC.forward): an ordinary logits tensor
    that routes ``F.cross_entropy(logits, labels)`` -- the reference closures'
    loss (citation.py:46-49, reddit.py:55-58), called unchanged -- to the HIP
    cross-entropy kernels (_LogitsCrossEntropy) instead of torch's one-
    workgroup nll reduction; any other form of the call and every other
    operation is torch's own and returns plain tensors.

    Only the direct form takes the HIP loss: F.cross_entropy(model(x), y)
    (or of the model's output object).  An indexed or otherwise transformed
    output -- F.cross_entropy(model(x)[idx], y) -- is a plain tensor, so that
    call is torch's own (same value to fp32 tolerance).  Labels are checked
    once per labels tensor (an out-of-range label raises IndexError, as torch
    fails on it)."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is F.cross_entropy:
            plain = _cross_entropy_args(args, kwargs)
            if plain is not None:
                x, y, ignore_index = plain
                return _LogitsCrossEntropy.apply(x.as_subclass(torch.Tensor), y, ignore_index)
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **kwargs)


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
        # (a logits tensor whose F.cross_entropy runs on the HIP kernels)
        return _LinearMFMA.apply(x, self.W.weight, self.W.bias).as_subclass(SGCLogits)


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
