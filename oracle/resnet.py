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

from . import dfxp, nn
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


def forward_backward(model, ranges, x, labels, step, seed, target=0.0, dz=None, norm=None):
    """Forward + loss + manual backward. Returns (loss, logits, grads, ctx).
    dz: d loss / d logits to back-propagate instead of the oracle's own (a test injects the GPU's:
    the softmax is the one op of the step that is not bit-exact, so with the same dz the whole
    backward and update are). norm: the batch the loss mean is over (data-parallel shards: global)."""
    ctx = nn.Ctx(ranges, step, seed, target)
    logits = model.forward(np.asarray(x, F32), ctx)
    loss, dz_own = nn.softmax_xent(logits, np.asarray(labels), norm)
    model.backward(dz_own if dz is None else np.asarray(dz, F32), ctx)
    ctx.logits, ctx.dz = logits, dz_own
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


def train_step(model, state, x, labels, lr=1e-2, momentum=0.9, seed=0, target=0.0, dz=None):
    """One ``Trainer.train`` batch (``trainer.py:157``) on the numpy model.

    ``state`` = dict(params, accum, ranges, step). Returns (loss, new_state, ctx).
    dz: injected d loss / d logits (see forward_backward).
    """
    set_params(model, state["params"])
    loss, logits, grads, ctx = forward_backward(model, state["ranges"], x, labels, state["step"], seed, target, dz)
    params, accum = sgd_momentum(state["params"], grads, state["accum"], lr, momentum)
    new_state = dict(params=params, accum=accum, ranges=ctx.new_ranges(), step=state["step"] + 1)
    return loss, new_state, ctx


def _walk(layer):
    yield layer
    for attr in ("layers", "residual", "shortcut"):
        sub = getattr(layer, attr, None)
        if sub is None:
            continue
        for s in (sub if isinstance(sub, list) else [sub]):
            yield from _walk(s)


def _numerators(model):
    """{param name: (kind, int64 numerator, scale, owner)} of the last backward: the integers each
    gradient is dequantised from (the data-parallel exchange sums exactly these)."""
    out = {}
    for layer in _walk(model):
        if isinstance(layer, (nn.Conv2dQ, nn.DenseQ)):
            out[layer.name + "/W"] = ("w", layer.acc_w, layer.ew_grad, layer)
        elif isinstance(layer, nn.RescaleQ):
            out[layer.name + "/g"] = ("g", layer.sgr, layer.sgsr, layer)
            out[layer.name + "/b"] = ("b", layer.sg, layer.eg, layer)
    return out


def dp_train_step(model, state, shards, lr=1e-2, momentum=0.9, seed=0, target=0.0, dzs=None):
    """One data-parallel step over batch shards [(x_r, labels_r)], each
    rank with its own batch statistics (standard DDP BatchNorm): every shard runs forward +
    backward with the loss normalised by the GLOBAL batch; the exact integer numerators of every
    weight / gamma / beta gradient and every quantiser's overflow counts are summed over the
    shards (the build's one int64 all-reduce) and dequantised once, with the formulas of the
    single-process step; then one SGD-momentum update and one range update from the summed
    counts. dzs: per-shard injected d loss / d logits. Returns (global loss, new_state, ctxs)."""
    B = sum(len(y) for _, y in shards)
    num, counts, loss, ctxs = None, {}, 0.0, []
    for r, (x, y) in enumerate(shards):
        set_params(model, state["params"])
        l, _, _, ctx = forward_backward(model, state["ranges"], x, y, state["step"], seed, target,
                                        None if dzs is None else dzs[r], norm=B)
        loss += l
        ctxs.append(ctx)
        nr = _numerators(model)
        if num is None:
            num = {k: [kind, v.astype(np.int64).copy(), sc, owner] for k, (kind, v, sc, owner) in nr.items()}
        else:
            for k, (_, v, _, _) in nr.items():
                num[k][1] = num[k][1] + v
        for name, (c1, c2, n, bits) in ctx.counts.items():
            a = counts.get(name, (0, 0, 0, bits))
            counts[name] = (a[0] + c1, a[1] + c2, a[2] + n, bits)
    grads = {}
    for k, (kind, S, sc, owner) in num.items():
        if kind == "w":
            grads[k] = (nn.scale_int(S, sc) + (F32(2 * owner.wd) * owner.W).astype(F32)).astype(F32)
        elif kind == "g":
            grads[k] = ((S.astype(np.float64) * sc).astype(F32) + (F32(2 * owner.wd) * owner.gamma).astype(F32)).astype(F32)
        else:
            grads[k] = (S.astype(np.float64) * sc).astype(F32)
    params, accum = sgd_momentum(state["params"], grads, state["accum"], lr, momentum)
    ranges = dict(state["ranges"])
    for name, (c1, c2, n, bits) in counts.items():
        ranges[name] = dfxp.update_range_from_counts(c1, c2, n, target, bits, state["ranges"][name])
    return loss, dict(params=params, accum=accum, ranges=ranges, step=state["step"] + 1), ctxs
