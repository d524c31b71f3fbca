"""``dfxp`` -- the PyTorch face the reference's ``custom.py`` imports
(``from .dfxp import Conv2d_q, Linear_q, BatchNorm2d_q``, ``custom.py:5``), backed by
``torch.autograd.Function``s over the gfx950 DFXP kernels. The TF-style Layer_q API is in
:mod:`lbt_amd.dynamic_fixed_point`.
"""
from .modules import BatchNorm2d_q, Conv2d_q, Linear_q, update_range_op  # noqa: F401

__all__ = ["Conv2d_q", "Linear_q", "BatchNorm2d_q", "update_range_op"]
