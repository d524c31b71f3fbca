"""Models of the reference (``models.py``) on the gfx950 DFXP layers.

``Model`` mirrors ``models.py:7-54``: it owns the layer list, runs the forward pass, the mean
sparse softmax cross-entropy (``:30-32``) and the manual backward from d loss / d logits through
``reversed(layers)`` (``:47-51``). ``CIFAR10_Resnet`` / ``CIFAR10_Resnet20/32/44/56`` mirror
``:371-470``. Inputs are NHWC fp32 CUDA tensors, labels int32.
"""
import torch

from . import dynamic_fixed_point as L
from .dfxp import ops
from .dfxp.layers import _Cache, backward_scope
from .runtime import default_context


def _lib_load():
    from . import _lib
    return _lib.load()


class Model:
    def __init__(self, bits, input_shape, dropout=0.5, weight_decay=0, stochastic=False, ctx=None):
        self.bits = bits
        self.input_shape = input_shape
        self.dropout = dropout
        self.weight_decay = weight_decay
        self.stochastic = stochastic
        self.ctx = ctx or default_context()
        self.training = True
        self.layers = self.get_layers()
        if self.layers and hasattr(self.layers[0], "need_input_grad"):
            self.layers[0].need_input_grad = False  # d loss / d input is never consumed
        self._c = _Cache()
        self.logits = None
        self.loss = None

    def get_layers(self):
        return []

    batched_params = True  # one launch for every weight quantiser, one for every gamma / beta

    def _walk(self):
        out = []

        def rec(layer):
            out.append(layer)
            for sub in getattr(layer, "layers", []):
                rec(sub)
            for attr in ("residual", "shortcut"):
                if hasattr(layer, attr):
                    rec(getattr(layer, attr))
        for layer in self.layers:
            rec(layer)
        return out

    def _build_param_prologue(self):
        """Job lists of the batched parameter quantisers (batched.hip): every conv / dense weight
        whose packed images need no column sums (the wide, LDS-tiled kernels' layers) and every
        Rescale_q gamma / beta -- bit-identical to each layer quantising its own."""
        from ._lib import OUT_F32, QJob, WJob
        from .fused import _dev_array
        wjobs, starts, qjobs = [], [0], []
        for layer in self._walk():
            if getattr(layer, "fmode", False):
                continue  # 17..32-bit layers quantise their own parameters as fp32 values
            if isinstance(layer, L.Conv2d_q) and not layer.mfma and not getattr(layer, "w4", False) \
                    and layer.ksize[3] % 4 == 0:
                kh, kw, ci, co = layer.ksize
                layer.W_range.observe(layer.W.numel())
                wjobs.append(WJob(layer.W.data_ptr(), kh, kw, ci, co, layer.W_range.desc, layer.w_hwio.data_ptr(),
                                  layer.wf.data_ptr() if layer.igemm_f else None, layer.ksf,
                                  layer.wd.data_ptr() if layer.igemm_d else None, layer.ksd, None))
            elif isinstance(layer, L.Dense_q) and layer.units % 4 == 0:
                layer.W_range.observe(layer.W.numel())
                wjobs.append(WJob(layer.W.data_ptr(), layer.in_units, 1, 1, layer.units, layer.W_range.desc,
                                  layer.w_hwio.data_ptr(), None, 0, None, 0, None))
            elif isinstance(layer, L.Rescale_q):
                C = layer.C
                layer.g_range.observe(C)
                layer.b_range.observe(C)
                qjobs.append(QJob(layer.gamma.data_ptr(), layer.gb.data_ptr(), OUT_F32, C, 1, layer.g_range.desc))
                qjobs.append(QJob(layer.beta.data_ptr(), layer.gb.data_ptr() + 4 * C, OUT_F32, C, 1,
                                  layer.b_range.desc))
            else:
                continue
            layer._batched_q = True
        lib = _lib_load()
        for j in wjobs:
            starts.append(starts[-1] + lib.lbt_flat_weight_blocks(j.KH * j.KW * j.Cin * j.Cout))
        dev = self.ctx.device
        self._pro = (_dev_array(wjobs, dev) if wjobs else None, len(wjobs),
                     torch.tensor(starts, dtype=torch.int32, device=dev), starts[-1],
                     _dev_array(qjobs, dev) if qjobs else None, len(qjobs))

    def _param_prologue(self):
        if getattr(self, "_pro", None) is None:
            self._build_param_prologue()
        wj, nw, starts, nb, qj, nq = self._pro
        if nw:
            ops.quantize_weights_flat(wj, starts, nw, nb)
        if nq:
            ops.quantize_many(qj, nq)
        self.ctx.params_ready = True

    def forward(self, X):
        self.ctx.fill_noise_tables()  # this step's noise of the quantisers that read tables
        if self.batched_params:
            self._param_prologue()
        try:
            for layer in self.layers:
                X = layer.forward(X)
        finally:
            self.ctx.params_ready = False
        self.logits = X
        return X

    def _norm_layers(self):
        return [l for l in self._walk() if isinstance(l, L.Normalization_q)]

    def set_testing(self):
        """models.py:15 ``set_testing``: every Normalization_q normalises with its running averages
        (dynamic_fixed_point.py:590-600). The layer-wise model only (a FusedResNet plan is built for
        training-mode BatchNorm, which is also what the reference's test loop runs, trainer.py:164)."""
        self.training = False
        for n in self._norm_layers():
            n.train = False

    def set_training(self):
        """models.py:14 ``set_training``."""
        self.training = True
        for n in self._norm_layers():
            n.train = True

    def compute_loss(self, labels):
        """loss = mean(sparse_softmax_cross_entropy(labels, logits)); keeps d loss / d logits."""
        z = self.logits
        self.loss = self._c.get("loss", (1,), torch.float32, z.device)
        self.dlogits = self._c.get("dz", z.shape, torch.float32, z.device)
        ops.softmax_xent(z, labels, self.loss, self.dlogits)
        return self.loss

    def accuracy(self, labels):
        return (self.logits.argmax(dim=1).to(torch.int32) == labels).float().mean()

    def backward(self):
        grad = self.dlogits
        with backward_scope():  # joins the weight / BN-parameter gradients launched on the side stream
            for layer in reversed(self.layers):
                grad = layer.backward(grad, self.stochastic)
        return grad

    def grads_and_vars(self):
        res = []
        for layer in self.layers:
            res += layer.grads_and_vars()
        return res

    def param_slots(self):
        return [s for layer in self.layers for s in layer.param_slots()]

    def info(self):
        return "\n".join([layer.info() for layer in self.layers])


class CIFAR10_Resnet(Model):
    def __init__(self, bits, num_blocks, block, dropout=0.5, weight_decay=0, stochastic=False, ctx=None,
                 weight_bits=None, grad_range=2):
        self.num_blocks = num_blocks
        self.block = block
        self.weight_bits = weight_bits  # config 5: 4-bit weights, 8-bit activations / gradients
        # the initial value of every layer's grad_range variable (the layers' own constructor argument,
        # dynamic_fixed_point.py:225,321,541,628; the reference builder leaves it at its default 2)
        self.grad_range = grad_range
        super().__init__(bits, [None, 32, 32, 3], dropout, weight_decay, stochastic, ctx)

    def _build_blocks(self, channels, num_blocks, stride):
        blocks = []
        for i in range(1, 1 + num_blocks):
            blocks.append(self.block(name="block%d-%d" % (channels, i), bits=self.bits, in_channels=self.channels,
                                     channels=channels, stride=1 if i > 1 else stride, training=self.training,
                                     weight_decay=self.weight_decay, weight_bits=self.weight_bits,
                                     grad_range=self.grad_range, ctx=self.ctx))
            self.channels = channels * self.block.expansion
        return blocks

    def get_layers(self):
        self.channels = 16
        return [
            L.Conv2d_pq(name="conv1", bits=self.bits, ksize=[3, 3, 3, 16], strides=[1, 1, 1, 1], padding="SAME",
                        use_bias=False, weight_decay=self.weight_decay, weight_bits=self.weight_bits,
                        grad_range=self.grad_range, ctx=self.ctx),
            L.BatchNorm_q(name="conv1-bn", bits=self.bits, num_features=16, training=self.training,
                          weight_decay=self.weight_decay, grad_range=self.grad_range, ctx=self.ctx),
            L.ReLU_q(),
        ] + self._build_blocks(16, self.num_blocks[0], 1) \
          + self._build_blocks(32, self.num_blocks[1], 2) \
          + self._build_blocks(64, self.num_blocks[2], 2) \
          + [
            L.AvgPool_q(ksize=[1, 8, 8, 1], strides=[1, 1, 1, 1], padding="VALID"),
            L.Flatten_q(64),
            L.Dense_q(name="softmax", bits=self.bits, in_units=64, units=10, use_bias=False,
                      weight_decay=self.weight_decay, weight_bits=self.weight_bits, grad_range=self.grad_range,
                      ctx=self.ctx),
        ]


def CIFAR10_Resnet20(bits, dropout=0.5, weight_decay=0, stochastic=False, ctx=None, weight_bits=None, grad_range=2):
    return CIFAR10_Resnet(bits, [3, 3, 3], L.ResidualBlock_q, dropout, weight_decay, stochastic, ctx, weight_bits,
                          grad_range)


def CIFAR10_Resnet32(bits, dropout=0.5, weight_decay=0, stochastic=False, ctx=None):
    return CIFAR10_Resnet(bits, [5, 5, 5], L.ResidualBlock_q, dropout, weight_decay, stochastic, ctx)


def CIFAR10_Resnet44(bits, dropout=0.5, weight_decay=0, stochastic=False, ctx=None):
    return CIFAR10_Resnet(bits, [7, 7, 7], L.ResidualBlock_q, dropout, weight_decay, stochastic, ctx)


def CIFAR10_Resnet56(bits, dropout=0.5, weight_decay=0, stochastic=False, ctx=None):
    return CIFAR10_Resnet(bits, [9, 9, 9], L.ResidualBlock_q, dropout, weight_decay, stochastic, ctx)


class ImageNet_Resnet(Model):
    """ResNet on ImageNet-shape inputs composed from ``ResidualBottleneck_q`` (``:878-980``) and
    ``MaxPool_q`` (``:993-1006``) -- the reference has both but no builder:
    conv 7x7/2 -> BN -> ReLU -> max pool 3x3/2 SAME -> stages of bottlenecks at width, 2w, 4w, 8w
    (strides 1, 2, 2, 2, the stride on the 3x3 as the reference block has it) -> global average
    pool -> flatten -> Dense_q. ``grad_bits`` sets every gradient quantiser's width (config 4: 16)."""

    def __init__(self, bits, num_blocks, grad_bits=None, width=64, classes=1000, image=224, weight_decay=0,
                 stochastic=False, ctx=None):
        self.num_blocks, self.grad_bits, self.width, self.classes = tuple(num_blocks), grad_bits, width, classes
        super().__init__(bits, [None, image, image, 3], 0.5, weight_decay, stochastic, ctx)

    def get_layers(self):
        c, gb, wd, ctx, bits = self.width, self.grad_bits, self.weight_decay, self.ctx, self.bits
        image = self.input_shape[1]
        layers = [
            L.Conv2d_pq(name="conv1", bits=bits, ksize=[7, 7, 3, c], strides=[1, 2, 2, 1], padding="SAME",
                        use_bias=False, weight_decay=wd, grad_bits=gb, ctx=ctx),
            L.BatchNorm_q(name="conv1-bn", bits=bits, num_features=c, training=self.training, weight_decay=wd,
                          grad_bits=gb, ctx=ctx),
            L.ReLU_q(),
            L.MaxPool_q(ksize=[1, 3, 3, 1], strides=[1, 2, 2, 1], padding="SAME"),
        ]
        in_ch = c
        for si, (nb, stride) in enumerate(zip(self.num_blocks, (1, 2, 2, 2))):
            ch = c << si
            for i in range(1, nb + 1):
                layers.append(L.ResidualBottleneck_q(name="block%d-%d" % (ch, i), bits=bits, in_channels=in_ch,
                                                     channels=ch, stride=stride if i == 1 else 1,
                                                     training=self.training, weight_decay=wd, grad_bits=gb, ctx=ctx))
                in_ch = 4 * ch
        hw = image
        for s in (2, 2, 1, 2, 2, 2):  # conv1, max pool, stage strides
            hw = -(-hw // s)
        layers[3].pool_relu = layers[2]  # the stem ReLU (forward and backward) runs inside the pool
        layers[2].act_in_pool = True
        blocks = [l for l in layers if isinstance(l, L.ResidualBottleneck_q)]
        for a, b in zip(blocks, blocks[1:]):
            a.next_block = b  # fused blocks hand their output's conv codes to the next block
            b.prev_block = a  # ... and their input gradient back as an unsummed pair
        layers += [
            L.AvgPool_q(ksize=[1, hw, hw, 1], strides=[1, 1, 1, 1], padding="VALID"),
            L.Flatten_q(in_ch),
            L.Dense_q(name="fc", bits=bits, in_units=in_ch, units=self.classes, use_bias=False, weight_decay=wd,
                      grad_bits=gb, ctx=ctx),
        ]
        return layers


def ImageNet_Resnet50(bits, grad_bits=None, weight_decay=0, classes=1000, image=224, width=64, ctx=None):
    return ImageNet_Resnet(bits, (3, 4, 6, 3), grad_bits, width, classes, image, weight_decay, ctx=ctx)
