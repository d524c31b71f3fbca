"""Data-parallel exchange of the DFXP training step (torch.distributed: RCCL on MI355X, gloo on CPU).

The reference is single-process (trainer.py:69-71). The build shards the batch over ranks (one
process per GPU) and adds ONE collective per step. For the fused plans (the bench path) it is an
all-reduce SUM of the int64 exchange buffer

    [ every gradient element's integer numerator (272 464 for ResNet-20) | overflow counters
      (2 per quantiser) | loss-term sum in 2^-32 fixed point ]

written by lbt_step_reduce_x at the end of the backward: the weight gradient of :302 is
dequant(sum_pixels Xq * Gq) + 2*wd*W, so summing the integer sums over ranks and dequantising once
(lbt_step_finish) is EXACT -- the quantised-gradient exchange of SURVEY 8(e) -- and independent of
the order RCCL adds in. (2.2 MB; latency-bound on xGMI, one flat bucket.)

Layer-wise models whose trainable variables are all integer-coded (quantised conv / dense W, BN
gamma / beta: exact_layerwise_ok -- the ResNet-50 of configs[3]) use the SAME int64 exchange: while
the Trainer runs their forward / backward, ops.set_exchange_sink points every gradient reduction
(lbt_conv_wgrad_reduce(64)_x, lbt_dense_wgrad_x, lbt_bn_param_grads_x) at the gradient's slots of the
buffer, the softmax (lbt_softmax_xent_n) normalises by the global batch and leaves its loss sum in the
loss slot, and lbt_step_reduce_x's fold blocks add the counters: an N-rank step equals the oracle's
N-shard step bit for bit (tests/test_dp_resnet50_gpu.py).

Other layer-wise models (fp32-mode layers, biases) exchange dequantised gradients instead, an
all-reduce SUM of

    [ flat fp32 gradients | every quantiser's folded overflow counters ]

The gradient buffer IS the head of the comm buffer (the backward writes into it), and the counter
fold kernel (lbt_dfxp_counts_fold) writes each slot's totals into the tail as exact fp32 pairs
(c >> 12, c & 4095: every partial sum of the all-reduce stays below 2**24), so the exchange is one
in-place RCCL call on ~1.1 MB -- latency-bound on xGMI, so a single flat bucket beats bucketing. After it,
every rank applies the same averaged update (SGD gscale = 1/world) and the same range update
(nelem = per-rank elements x world), i.e. the DFXP exponents stay identical on all ranks without
any extra synchronisation. The rounding-noise key (seed, step, quantiser) does not involve the
rank, so activation noise (shape X.shape[1:]) is what a single process would draw.
"""
import torch
import torch.distributed as dist

FOLD = 4  # floats per quantiser slot in the comm buffer tail


def make_comm_buffer(n_grads, n_slots, device):
    """[grads | FOLD floats per quantiser slot] fp32."""
    return torch.zeros(n_grads + FOLD * n_slots, dtype=torch.float32, device=device)


def fold_host(c):
    """Host twin of lbt_dfxp_counts_fold's packing: int [slots, 2] -> fp32 [slots*4]."""
    c = torch.as_tensor(c, dtype=torch.int64).view(-1, 2)
    return torch.stack([c[:, 0] >> 12, c[:, 0] & 4095, c[:, 1] >> 12, c[:, 1] & 4095], 1).float().view(-1)


def unfold_host(f):
    """fp32 [slots*4] -> int64 [slots, 2] (what lbt_dfxp_range_update_folded decodes)."""
    f = f.view(-1, 4).to(torch.int64)
    return torch.stack([f[:, 0] * 4096 + f[:, 1], f[:, 2] * 4096 + f[:, 3]], 1)


def make_exchange(n_grads, n_slots, device):
    """The int64 exchange buffer [numerators | 2 counters per slot | loss] and its lbt_xchg
    descriptor (buf, cnt_off, loss_off, nslots set; the caller sets gbase / counts / pjob_scale)."""
    from . import _lib
    buf = torch.zeros(n_grads + 2 * n_slots + 1, dtype=torch.int64, device=device)
    x = _lib.Xchg()
    x.buf = buf.data_ptr()
    x.nslots = n_slots
    x.cnt_off = n_grads
    x.loss_off = n_grads + 2 * n_slots
    x.pjob_scale = 1
    return buf, x


def finish_segments(flat, device):
    """lbt_fseg per parameter tensor of a FlatParams (kind 0 conv / dense W, 1 gamma, 2 beta) as a
    device array (raw bytes), and the finish kernel's block count."""
    from . import _lib
    from .dfxp import ops
    segs, blocks = [], 0
    for owner, var, off, sz in flat.offsets:
        if var == "W":
            kind, qx, qg = 0, owner.X_range.desc, owner.grad_range.desc
        elif var == "gamma":
            kind, qx, qg = 1, owner.X_range.desc, owner.grad_range.desc
        elif var == "beta":
            kind, qx, qg = 2, owner.X_range.desc, owner.grad_range.desc
        else:
            raise NotImplementedError("exact exchange of parameter %r" % var)
        segs.append(_lib.FSeg(off, sz, kind, qx, qg, ops.f32(2 * owner.weight_decay)))
        blocks += (sz + 255) // 256
    raw = bytes((_lib.FSeg * len(segs))(*segs))
    return torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device), blocks


def exact_layerwise_ok(model):
    """True when every trainable variable of a layer-wise model gets an INTEGER gradient numerator
    (quantised conv / dense W, BN gamma / beta; no fp32-mode layer, no bias): the models the exact
    int64 exchange (ops.set_exchange_sink) takes."""
    for owner, var, _ in model.param_slots():
        if var not in ("W", "gamma", "beta") or getattr(owner, "fmode", False):
            return False
    return True


def allreduce_comm(comm, group=None):
    """The step's only collective: in-place SUM of [grads | folded counters] over the ranks."""
    dist.all_reduce(comm, op=dist.ReduceOp.SUM, group=group)
