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
"""
import itertools

import torch
from torch import nn

from ..runtime import default_context
from . import layers as L

_ids = itertools.count()


def update_range_op(ctx=None):
    (ctx or default_context()).update_range_op()


class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x, weight, bias, mod):
        mod._load_params(weight, bias)
        y = mod.layer.forward(x.contiguous())
        fctx.mod = mod
        return y.clone()

    @staticmethod
    def backward(fctx, gy):
        mod = fctx.mod
        dx = mod.layer.backward(gy.contiguous(), True).clone()
        dw, db = mod._param_grads()
        return dx, dw, db, None


class Conv2d_q(nn.Module):
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


class Linear_q(nn.Module):
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
        mod.rescale.gamma.copy_(gamma.detach())
        mod.rescale.beta.copy_(beta.detach())
        y = mod.rescale.forward(mod.norm.forward(x.contiguous()))
        fctx.mod = mod
        return y.clone()

    @staticmethod
    def backward(fctx, gy):
        mod = fctx.mod
        g = mod.rescale.backward(gy.contiguous(), True)
        dx = mod.norm.backward(g, True).clone()
        return dx, mod.rescale.dgamma.clone(), mod.rescale.dbeta.clone(), None


class BatchNorm2d_q(nn.Module):
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
