"""lbt_amd -- MI355X-native dynamic fixed point (DFXP) low-bit training.

A from-scratch gfx950 implementation of the hot path of freudh/lbt: the DFXP quantiser and
overflow-rate range controller, the quantised conv / dense / batch-norm forward and backward on
int8 MFMA implicit GEMMs, and data-parallel ResNet training over RCCL.

* :mod:`lbt_amd.dynamic_fixed_point` -- the reference's TF-face API (Layer_q classes)
* :mod:`lbt_amd.dfxp`                -- the PyTorch face (Conv2d_q / Linear_q / BatchNorm2d_q)
* :mod:`lbt_amd.models`              -- CIFAR10_Resnet20/32/44/56
* :mod:`lbt_amd.trainer`             -- the training step (HIP-graph captured, RCCL data parallel)
"""
from .runtime import DfxpContext, default_context, set_default_context  # noqa: F401
