"""PyTorch nn.Module face of the DFXP layers -- the names ``custom.py:5`` imports.

``Conv2d_q(bits, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=False)``
(``custom.py:10-12``), ``Linear_q(bits, in_features, out_features, bias=True)``
(``custom.py:29-30``) and ``BatchNorm2d_q(bits, num_features)`` (imported at ``custom.py:5``;
the reference never shows its signature, so the torch convention is adopted).

Each module wraps the corresponding Layer_q of :mod:`lbt_amd.dfxp.layers` in a
``torch.autograd.Function``: forward quantises input / weight and runs the integer GEMM,
backward quantises the incoming gradient and returns dX and dW (straight-through estimator:
the gradient passes the quantiser unchanged, ``dynamic_fixed_point.py:30,38``).
Tensors use torch's logical NCHW shapes; internally they are NHWC (channels_last) because
that is the layout the kernels stream. Weight decay belongs to the torch optimiser here.
Call :func:`update_range_op` after each optimiser step (the reference's ``'update_range'``
collection).

Module reuse. A Layer_q keeps what its backward needs (input codes, BN moments, Rescale codes) on
the layer itself, in buffers the next forward overwrites -- the reference's TF ``Layer_q`` has the
same single-use assumption (``dynamic_fixed_point.py:97-126``). PyTorch users expect a module to be
callable several times per graph, so each call holds a token; when a call's state is about to be
overwritten while its autograd graph is still alive, the state is snapshotted into that call's token,
and restored into the layer before that call's backward (in whatever order autograd runs them).
Single-use modules never snapshot (no copies on the common path).
"""
import itertools
import weakref

import torch
from torch import nn

from ..runtime import default_context
from . import layers as L

_ids = itertools.count()

# what each Layer_q's backward reads from its own forward (beyond parameters and quantisers,
# which do not change within a step): X is the caller's tensor (kept by reference), the rest are
# layer-owned buffers a later forward rewrites
_STATE = {
    L.Conv2d_q: ("X", "xq", "wq", "d"),
    L.Dense_q: ("X", "xq", "wq", "d"),
    L.Normalization_q: ("X", "q", "n", "ms"),
    L.Rescale_q: ("X", "R", "xr"),
}


def update_range_op(ctx=None):
    (ctx or default_context()).update_range_op()


class _Call:
    """One forward call of a module: the layers' state it produced once a later call displaced it."""
    __slots__ = ("snap", "__weakref__")

    def __init__(self):
        self.snap = None


def _snapshot(layers):
    out = []
    for layer in layers:
        s = {}
        for a in _STATE[type(layer)]:
            if hasattr(layer, a):
                v = getattr(layer, a)
                s[a] = v.clone() if (torch.is_tensor(v) and a != "X") else v
        out.append(s)
    return out


def _restore(layers, snap):
    for layer, s in zip(layers, snap):
        for a, v in s.items():
            cur = getattr(layer, a, None)
            if (a != "X" and torch.is_tensor(v) and torch.is_tensor(cur) and cur.shape == v.shape
                    and cur.dtype == v.dtype and cur.device == v.device):
                cur.copy_(v)  # the layer's own buffer (descriptors may hold its address)
            else:
                setattr(layer, a, v)


def _begin_forward(mod):
    """Called before a forward overwrites the layers' state: a still-live earlier call keeps a copy."""
    prev = mod._owner() if mod._owner is not None else None
    if prev is not None and prev.snap is None:
        prev.snap = _snapshot(mod._layers())
    call = _Call()
    mod._owner = weakref.ref(call)
    return call


def _begin_backward(mod, call):
    """Called before a backward reads the layers' state: make it this call's."""
    cur = mod._owner() if mod._owner is not None else None
    if cur is call:
        return
    if call.snap is None:  # pragma: no cover - every displaced live call was snapshotted
        raise RuntimeError("%s: the forward state of this call was lost" % type(mod).__name__)
    if cur is not None and cur.snap is None:
        cur.snap = _snapshot(mod._layers())
    _restore(mod._layers(), call.snap)
    mod._owner = weakref.ref(call)


class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x, weight, bias, mod):
        fctx.call = _begin_forward(mod)
        mod._load_params(weight, bias)
        y = mod.layer.forward(x.contiguous())
        fctx.mod = mod
        return y.clone()

    @staticmethod
    def backward(fctx, gy):
        mod = fctx.mod
        _begin_backward(mod, fctx.call)
        dx = mod.layer.backward(gy.contiguous(), True).clone()
        dw, db = mod._param_grads()
        return dx, dw, db, None


class _Reusable(nn.Module):
    _owner = None

    def _layers(self):
        return (self.layer,)


class Conv2d_q(_Reusable):
    def __init__(self, bits, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=False, ctx=None,
                 name=None, input_nonnegative=False):
        super().__init__()
        k = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        s = (stride, stride) if isinstance(stride, int) else tuple(stride)
        self.layer = L.Conv2d_q(name or "Conv2d_q_%d" % next(_ids), bits, [k[0], k[1], in_channels, out_channels],
                                [1, s[0], s[1], 1], padding, use_bias=bias, weight_decay=0,
                                input_nonnegative=input_nonnegative, ctx=ctx)
        # torch layout [out, in, kh, kw]
        self.weight = nn.Parameter(self.layer.W.detach().permute(3, 2, 0, 1).contiguous())
        self.bias = nn.Parameter(torch.zeros(out_channels, device=self.layer.W.device)) if bias else None

    def _load_params(self, weight, bias):
        self.layer.W.copy_(weight.detach().permute(2, 3, 1, 0))
        if bias is not None:
            self.layer.b.copy_(bias.detach())

    def _param_grads(self):
        dw = self.layer.dW.permute(3, 2, 0, 1).contiguous()
        db = self.layer.db.clone() if self.bias is not None else None
        return dw, db

    def forward(self, x):
        y = _LayerFn.apply(x.permute(0, 2, 3, 1), self.weight, self.bias, self)
        return y.permute(0, 3, 1, 2)


class Linear_q(_Reusable):
    def __init__(self, bits, in_features, out_features, bias=True, ctx=None, name=None):
        super().__init__()
        self.layer = L.Dense_q(name or "Linear_q_%d" % next(_ids), bits, in_features, out_features, use_bias=bias,
                               weight_decay=0, ctx=ctx)
        self.weight = nn.Parameter(self.layer.W.detach().t().contiguous())  # torch [out, in]
        self.bias = nn.Parameter(torch.zeros(out_features, device=self.layer.W.device)) if bias else None

    def _load_params(self, weight, bias):
        self.layer.W.copy_(weight.detach().t())
        if bias is not None:
            self.layer.b.copy_(bias.detach())

    def _param_grads(self):
        return self.layer.dW.t().contiguous(), (self.layer.db.clone() if self.bias is not None else None)

    def forward(self, x):
        return _LayerFn.apply(x, self.weight, self.bias, self)


class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x, gamma, beta, mod):
        fctx.call = _begin_forward(mod)
        mod.rescale.gamma.copy_(gamma.detach())
        mod.rescale.beta.copy_(beta.detach())
        y = mod.rescale.forward(mod.norm.forward(x.contiguous()))
        fctx.mod = mod
        return y.clone()

    @staticmethod
    def backward(fctx, gy):
        mod = fctx.mod
        _begin_backward(mod, fctx.call)
        g = mod.rescale.backward(gy.contiguous(), True)
        dx = mod.norm.backward(g, True).clone()
        return dx, mod.rescale.dgamma.clone(), mod.rescale.dbeta.clone(), None


class BatchNorm2d_q(_Reusable):
    def _layers(self):
        return (self.norm, self.rescale)

    def __init__(self, bits, num_features, momentum=0.999, eps=1e-5, ctx=None, name=None):
        super().__init__()
        name = name or "BatchNorm2d_q_%d" % next(_ids)
        self.norm = L.Normalization_q(name + "-norm", bits, num_features, True, momentum, eps, ctx=ctx)
        self.rescale = L.Rescale_q(name + "-rescale", bits, num_features, weight_decay=0, ctx=ctx)
        self.weight = nn.Parameter(self.rescale.gamma.detach().clone())
        self.bias = nn.Parameter(self.rescale.beta.detach().clone())

    def forward(self, x):
        y = _BNFn.apply(x.permute(0, 2, 3, 1), self.weight, self.bias, self)
        return y.permute(0, 3, 1, 2)
