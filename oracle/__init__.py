"""CPU oracle for the DFXP training hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, in numpy, the semantics of the reference's dynamic
fixed point (DFXP) path so the HIP path can be checked against it:

* ``philox``   -- Philox4x32-10 counter RNG (the build's noise source; pinned by
                  the Random123 published known-answer vectors).
* ``dfxp``     -- ``weight_quantization`` / ``overflow_rate`` / ``update_range``
                  (reference ``dynamic_fixed_point.py:4-94``).
* ``nn``       -- the quantised layers' forward/backward
                  (reference ``dynamic_fixed_point.py:97-1053``).
* ``resnet``   -- ``CIFAR10_Resnet20`` + one ``Trainer`` step
                  (reference ``models.py:7-54,371-455``, ``trainer.py:79-84,144-162``).

Import rules (enforced by review, see DESIGN.md "Oracle"): only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / CPU baseline. The product path
(``lbt_amd``) never imports it and has no CPU fallback.

Pinning: the reference is TensorFlow 1.x graph code with no tests and cannot be
run here (TensorFlow absent, no network). The quantiser/controller restatement
is pinned by hand-derived known-answer vectors computed from the reference
formulas (``tests/golden/kat_dfxp.json``, derivations in SURVEY.md section 4);
the layer/model restatement follows the cited reference lines and is
"partially pinned" (formula-level KATs only). TF's own Philox stream cannot be
reproduced, so stochastic rounding parity is defined on the build's counter RNG
(same noise on CPU and GPU) -- see DESIGN.md.
"""
