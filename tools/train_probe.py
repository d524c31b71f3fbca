"""Training-dynamics probe: does the DFXP ResNet-20 step learn, and what
drives the loss blow-up on the bench's random-label batches?

    python tools/train_probe.py [--steps 300] [--out gpurun_out/train_probe.json]

Runs on cuda:0 through the fused HIP plan (graph replay), the reference hyperparameters (lr 1e-2,
momentum 0.9, wd 2e-4, every range variable starting at I = 2):

* ``learnable``: 10 fixed random class templates T_c (32x32x3, |T| <= 1); x = 0.6 T_y + 0.4 U(-1,1)
  noise, fresh noise and labels every step -- the label is a function of the input's template;
  loss every step, then held-out accuracy through Trainer.evaluate;
* ``random``: the bench's 4 random-label batches cycled (bench.synthetic_batches), with the
  exponent trajectory of every quantiser family, to locate the walk that precedes divergence.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_trainer(seed, B, lr=1e-2, momentum=0.9, grad_i0=None):
    from lbt_amd.fused import FusedResNet
    from lbt_amd.models import CIFAR10_Resnet20
    from lbt_amd.runtime import DfxpContext
    from lbt_amd.trainer import Trainer
    ctx = DfxpContext(device="cuda:0", seed=seed)
    gm = CIFAR10_Resnet20(8, weight_decay=2e-4, ctx=ctx)
    if grad_i0 is not None:  # the reference's grad_range constructor argument (default 2) for every layer
        for q in ctx.quantizers:
            if q.name.endswith("/grad_range"):
                ctx.exps[q.slot] = grad_i0
    return ctx, gm, Trainer(FusedResNet(gm), lr=lr, momentum=momentum, batch_size=B, use_graph=True)


def templates(seed):
    g = np.random.default_rng(seed)
    return g.uniform(-1, 1, size=(10, 32, 32, 3)).astype(np.float32)


def learnable_batch(T, B, rng):
    y = rng.integers(0, 10, size=B).astype(np.int32)
    x = (0.6 * T[y] + 0.4 * rng.uniform(-1, 1, size=(B, 32, 32, 3))).astype(np.float32)
    return x, y


def family(name):
    """'block16-1-bn1-norm/grad_range' -> 'bn-norm/grad_range', 'block16-1-1/W_range' -> 'conv/W_range'."""
    layer, kind = name.rsplit("/", 1)
    if layer.endswith("-norm"):
        return "bn-norm/" + kind
    if layer.endswith("-rescale"):
        return "bn-rescale/" + kind
    if layer == "softmax":
        return "dense/" + kind
    return "conv/" + kind


def run_learnable(steps, B=128, seed=5, grad_i0=None):
    ctx, gm, tr = make_trainer(seed, B, grad_i0=grad_i0)
    T = templates(seed)
    rng = np.random.default_rng(seed)
    bufs = [(torch.empty((B, 32, 32, 3), device="cuda:0"), torch.empty((B,), dtype=torch.int32, device="cuda:0"))
            for _ in range(2)]
    losses = []
    for i in range(steps):
        x, y = learnable_batch(T, B, rng)
        X, Y = bufs[i % 2]
        X.copy_(torch.from_numpy(x))
        Y.copy_(torch.from_numpy(y))
        losses.append(float(tr.step(X, Y).item()))
    xt, yt = learnable_batch(T, 1000, np.random.default_rng(seed + 1))
    acc, tloss = tr.evaluate(xt, yt, batch_size=500)
    return dict(losses=losses, test_acc=acc, test_loss=tloss)


def run_random(steps, B=128, seed=1000, grad_i0=None):
    from bench import synthetic_batches
    ctx, gm, tr = make_trainer(0, B, grad_i0=grad_i0)
    xs, ys = synthetic_batches(4, B, seed, "cuda:0")
    names = [q.name for q in ctx.quantizers]
    losses, fams = [], {}
    for i in range(steps):
        losses.append(float(tr.step(xs[i % 4], ys[i % 4]).item()))
        r = ctx.ranges()
        for n in names:
            fams.setdefault(family(n), []).append(r[n])
    # per family: mean exponent per step
    traj = {f: np.asarray(v, np.float64).reshape(steps, -1).mean(1).round(2).tolist() for f, v in fams.items()}
    wmax = float(tr.flat.w.abs().max().item())
    return dict(losses=losses, exponent_mean_by_family=traj, final_max_abs_weight=wmax)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--random-steps", type=int, default=40)
    ap.add_argument("--batches", default="32,128")
    ap.add_argument("--grad-i0", default="2,-6", help="initial grad_range values to compare")
    ap.add_argument("--out", default="gpurun_out/train_probe.json")
    a = ap.parse_args()
    out = {}
    for gi in [int(v) for v in a.grad_i0.split(",")]:
        for B in [int(b) for b in a.batches.split(",")]:
            out["learnable_b%d_gI%d" % (B, gi)] = run_learnable(a.steps, B, grad_i0=gi)
            out["random_b%d_gI%d" % (B, gi)] = run_random(a.random_steps, B, grad_i0=gi)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, v in out.items():
        L = v["losses"]
        print("%-22s loss %.3f -> %.3f (mean of last 20 %.3f)%s" % (k, L[0], L[-1], float(np.mean(L[-20:])),
              ", test acc %.3f" % v["test_acc"] if "test_acc" in v else ""))


if __name__ == "__main__":
    main()
