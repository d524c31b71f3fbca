"""Data-parallel exchange of the DFXP training step (torch.distributed: RCCL on MI355X, gloo on CPU).

The reference is single-process (trainer.py:69-71). The build shards the batch over ranks (one
process per GPU) and adds ONE collective per step: an all-reduce SUM of

    [ flat fp32 gradients (272 464 for ResNet-20) | every quantiser's folded overflow counters ]

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


def allreduce_comm(comm, group=None):
    """The step's only collective: in-place SUM of [grads | folded counters] over the ranks."""
    dist.all_reduce(comm, op=dist.ReduceOp.SUM, group=group)
