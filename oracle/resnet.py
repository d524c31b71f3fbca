"""CIFAR-10 ResNet-20 and one training step, numpy (oracle; test infrastructure only).

Restates ``models.py:371-455`` (``CIFAR10_Resnet`` / ``CIFAR10_Resnet20``: conv1
(``Conv2d_pq``) -> BN -> ReLU -> 3 stages of ``ResidualBlock_q`` at 16/32/64
channels, strides 1/2/2 -> 8x8 average pool -> flatten -> ``Dense_q`` 64->10),
``models.py:27-51`` (mean sparse softmax cross-entropy; manual backward from
d loss / d logits through ``reversed(layers)``) and the timed step of
``trainer.py:144-162`` (``MomentumOptimizer``: ``acc = mu*acc + g; w -= lr*acc``,
``trainer.py:79-84``, fetched together with the ``update_range`` collection).
"""
import numpy as np

from . import nn
from .nn import F32


def build_resnet(num_blocks=(3, 3, 3), bits=8, weight_decay=0.0, weight_bits=None):
    """weight_bits: the weight quantisers' width (config 5: 4)."""
    wb = dict(weight_bits=weight_bits)
    layers = [nn.Conv2dQ("conv1", bits, [3, 3, 3, 16], [1, 1, 1, 1], "SAME", weight_decay, **wb),
              nn.BatchNormQ("conv1-bn", bits, 16, weight_decay),
              nn.ReluQ()]
    in_ch = 16
    for channels, nb, stride in zip((16, 32, 64), num_blocks, (1, 2, 2)):
        for i in range(1, nb + 1):
            layers.append(nn.ResidualBlockQ("block%d-%d" % (channels, i), bits, in_ch, channels,
                                            stride if i == 1 else 1, weight_decay, **wb))
            in_ch = channels
    layers += [nn.AvgPoolQ(), nn.FlattenQ(64), nn.DenseQ("softmax", bits, 64, 10, weight_decay, **wb)]
    return nn.SequentialQ(*layers)


def build_resnet50(blocks=(3, 4, 6, 3), width=64, classes=1000, bits=8, grad_bits=None, weight_decay=0.0):
    """ResNet-50 composed from ``ResidualBottleneck_q`` (the reference has the block, ``:878-980``,
    and ``MaxPool_q``, ``:993-1006``, but no builder): conv 7x7/2 -> BN -> ReLU -> max pool 3x3/2
    SAME -> 4 stages of bottlenecks at width, 2w, 4w, 8w (strides 1, 2, 2, 2; the stride on the 3x3,
    as the reference block has it) -> global average pool -> flatten -> Dense_q. grad_bits: the
    gradient quantisers' width (config 4: 16)."""
    gb = dict(grad_bits=grad_bits)
    layers = [nn.Conv2dQ("conv1", bits, [7, 7, 3, width], [1, 2, 2, 1], "SAME", weight_decay, **gb),
              nn.BatchNormQ("conv1-bn", bits, width, weight_decay, **gb),
              nn.ReluQ(),
              nn.MaxPoolQ([1, 3, 3, 1], [1, 2, 2, 1], "SAME")]
    in_ch = width
    for si, (nb, stride) in enumerate(zip(blocks, (1, 2, 2, 2))):
        ch = width << si
        for i in range(1, nb + 1):
            layers.append(nn.BottleneckQ("block%d-%d" % (ch, i), bits, in_ch, ch, stride if i == 1 else 1,
                                         weight_decay, **gb))
            in_ch = 4 * ch
    layers += [nn.AvgPoolQ(), nn.FlattenQ(in_ch), nn.DenseQ("fc", bits, in_ch, classes, weight_decay, **gb)]
    return nn.SequentialQ(*layers)


def param_list(model):
    """[(name, owner)] in grads_and_vars order."""
    return model.params()


def get_params(model):
    out = {}
    for name, owner in model.params():
        out[name] = _get(owner, name)
    return out


def _get(owner, name):
    if name.endswith("/W"):
        return owner.W
    if name.endswith("/g"):
        return owner.gamma
    return owner.beta


def set_params(model, params):
    for name, owner in model.params():
        v = np.asarray(params[name], dtype=F32).copy()
        if name.endswith("/W"):
            owner.W = v
        elif name.endswith("/g"):
            owner.gamma = v
        else:
            owner.beta = v


def get_grads(model):
    out = {}
    for name, owner in model.params():
        if name.endswith("/W"):
            out[name] = owner.dW
        elif name.endswith("/g"):
            out[name] = owner.dgamma
        else:
            out[name] = owner.dbeta
    return out


def init_ranges(model, initial=2):
    return {r: initial for r in model.range_names()}


def forward_backward(model, ranges, x, labels, step, seed, target=0.0):
    """Forward + loss + manual backward. Returns (loss, logits, grads, ctx)."""
    ctx = nn.Ctx(ranges, step, seed, target)
    logits = model.forward(np.asarray(x, F32), ctx)
    loss, dz = nn.softmax_xent(logits, np.asarray(labels))
    model.backward(dz, ctx)
    return loss, logits, get_grads(model), ctx


def sgd_momentum(params, grads, accum, lr, momentum):
    """TF MomentumOptimizer (use_nesterov=False), fp32, no FMA contraction."""
    lr = F32(lr)
    mu = F32(momentum)
    new_p, new_a = {}, {}
    for k in params:
        a = ((mu * accum[k]).astype(F32) + grads[k]).astype(F32)
        new_a[k] = a
        new_p[k] = (params[k] - (lr * a).astype(F32)).astype(F32)
    return new_p, new_a


def train_step(model, state, x, labels, lr=1e-2, momentum=0.9, seed=0, target=0.0):
    """One ``Trainer.train`` batch (``trainer.py:157``) on the numpy model.

    ``state`` = dict(params, accum, ranges, step). Returns (loss, new_state, ctx).
    """
    set_params(model, state["params"])
    loss, logits, grads, ctx = forward_backward(model, state["ranges"], x, labels, state["step"], seed, target)
    params, accum = sgd_momentum(state["params"], grads, state["accum"], lr, momentum)
    new_state = dict(params=params, accum=accum, ranges=ctx.new_ranges(), step=state["step"] + 1)
    return loss, new_state, ctx
