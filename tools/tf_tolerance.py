"""How far the reference's fp32 arithmetic lands from the build's exact arithmetic, along the bench
workload (ResNet-20, 8-bit DFXP, B=128, the bench's synthetic batches): oracle/tfarith.py.

    python tools/tf_tolerance.py [--steps 20] [--batch 128] [--grad-range -6] [--out FILE]

The HIP path equals the exact oracle bit for bit (tests/test_gpu_parity.py), so these numbers are
also the distance between the MI355X results and the reference's arithmetic."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import tfarith  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--grad-range", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import bench
    xs, ys = bench.synthetic_batches(4, a.batch, seed=1000, device="cpu")
    batches = [(x.numpy(), y.numpy()) for x, y in zip(xs, ys)]
    t0 = time.time()

    def log(m):
        print(json.dumps({k: (round(v, 9) if isinstance(v, float) else v) for k, v in m.items()
                          if k not in ("exponent_mismatch_names", "op_level", "control_tf32seq_vs_tf32")}), flush=True)
        c = m["control_tf32seq_vs_tf32"]
        print("  control " + json.dumps({k: float("%.3g" % c[k]) for k in ("loss_rel", "grad_rel_l2", "code_flips",
                                                                            "exponent_mismatches")}), flush=True)
        print("  op_level " + json.dumps({k: float("%.3g" % v) for k, v in m["op_level"].items()}), flush=True)
    res = tfarith.run(batches, a.steps, grad_range=a.grad_range, log=log)
    keys = ("loss_rel", "logits_rel", "grad_rel_max", "grad_rel_l2", "weights_rel_max", "bn_mean_rel_max",
            "bn_var_rel_max")
    summ = {k: float(max(m[k] for m in res)) for k in keys}
    summ.update(code_flips_per_step_max=max(m["code_flips"] for m in res),
                code_flip_fraction_max=max(m["code_flips"] / m["code_elems"] for m in res),
                exponent_mismatches_total=sum(m["exponent_mismatches"] for m in res),
                rates_equal_counts=all(m["rates_equal_counts"] for m in res))
    csum = {k: float(max(m["control_tf32seq_vs_tf32"][k] for m in res)) for k in keys}
    csum.update(code_flip_fraction_max=max(m["control_tf32seq_vs_tf32"]["code_flips"] / m["control_tf32seq_vs_tf32"]["code_elems"]
                                           for m in res),
                exponent_mismatches_total=sum(m["control_tf32seq_vs_tf32"]["exponent_mismatches"] for m in res))
    summ["control_tf32seq_vs_tf32"] = csum
    ops = {}
    for m in res:
        for k, v in m["op_level"].items():
            ops[k] = max(ops.get(k, 0.0), v)
    summ["op_level"] = ops
    doc = dict(workload="ResNet-20 CIFAR-10 8-bit DFXP, B=%d, bench synthetic batches (seed 1000), %d steps, "
                        "teacher-forced along the exact trajectory" % (a.batch, a.steps),
               grad_range=a.grad_range, model="oracle.nn ARITH='tf32' (fp32 sgemm + pairwise fp32 reductions) vs 'exact'",
               max=summ, steps=res, seconds=round(time.time() - t0, 1))
    print(json.dumps({"max": summ}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
