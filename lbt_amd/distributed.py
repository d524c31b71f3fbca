"""Data-parallel exchange of the DFXP training step (torch.distributed: RCCL on MI355X, gloo on CPU).

The reference is single-process (trainer.py:69-71). The build shards the batch over ranks (one
process per GPU) and adds ONE collective per step: an all-reduce SUM of

    [ flat fp32 gradients (272 464 for ResNet-20) | every quantiser's overflow counters ]

Counters are integers < 2**24 per step, so they travel exactly as fp32 in the same buffer (one
RCCL call, ~1.1 MB: latency-bound on xGMI, so a single flat bucket beats bucketing). After it,
every rank applies the same averaged update (SGD gscale = 1/world) and the same range update
(nelem = per-rank elements x world), i.e. the DFXP exponents stay identical on all ranks without
any extra synchronisation. The rounding-noise key (seed, step, quantiser) does not involve the
rank, so activation noise (shape X.shape[1:]) is what a single process would draw.
"""
import torch
import torch.distributed as dist


def make_comm_buffer(n_grads, n_counts, device):
    return torch.zeros(n_grads + n_counts, dtype=torch.float32, device=device)


def allreduce_grads_and_counts(flat_g, counts, comm, group=None):
    """Sum flat_g (fp32) and counts (int32) across ranks in one all-reduce, in place."""
    n = flat_g.numel()
    if comm.numel() != n + counts.numel():
        raise ValueError("comm buffer size mismatch")
    comm[:n].copy_(flat_g)
    comm[n:].copy_(counts)
    dist.all_reduce(comm, op=dist.ReduceOp.SUM, group=group)
    flat_g.copy_(comm[:n])
    counts.copy_(comm[n:])
