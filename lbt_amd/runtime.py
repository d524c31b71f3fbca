"""Device-resident DFXP state: the build's counterpart of the reference's range variables.

In the reference every quantised tensor has an int32 TF variable ``<layer>/<X|W|grad|...>_range``
(the integer bits I, ``dynamic_fixed_point.py:161-171,256-266,...``) and
``weight_quantization`` adds an ``update_range`` op to the graph collection
``'update_range'`` (``:40-41``) that the trainer fetches with every step
(``trainer.py:63,157``).

Here one ``DfxpContext`` owns, in device memory,
  exps   int32 [capacity]                 I per quantiser slot
  counts int32 [capacity, NSHARD, CSTRIDE] overflow counters accumulated by the kernels
                                         (2 used per shard; one cache line per shard)
  step   int64 [1]                        noise counter (incremented by every range update)
  bits / target / nelem                   per-slot controller constants
and ``update_range_op()`` is the collection: ONE kernel that applies update_range to every
slot. Nothing is read back to the host during a step, so a whole step can be captured in a
HIP graph.
"""
import zlib

import torch

from . import _lib
from ._lib import CSTRIDE, NSHARD, QDesc


def qid_of(name):
    """Stable 31-bit noise-stream id of a quantiser, from its range variable's name."""
    return zlib.crc32(name.encode("utf-8")) & 0x7FFFFFFF


class Quantizer:
    """One DFXP quantiser slot: name, bits, rounding mode; its I lives in ``ctx.exps[slot]``."""

    def __init__(self, ctx, name, slot, bits, stochastic, target):
        self.ctx, self.name, self.slot, self.bits = ctx, name, slot, int(bits)
        self.stochastic, self.target = bool(stochastic), float(target)
        self.qid = qid_of(name)
        self._nelem = None
        self._desc = None

    @property
    def desc(self):
        if self._desc is None:
            c = self.ctx
            self._desc = QDesc(c.exps.data_ptr(), c.counts.data_ptr(), c.step.data_ptr(), c.seed, self.qid,
                               self.slot, self.bits, 1 if self.stochastic else 0)
        return self._desc

    def desc_nostats(self):
        d = QDesc.from_buffer_copy(self.desc)
        d.counts = None
        return d

    def observe(self, nelem):
        """Declare how many elements this quantiser sees per step (update_range's mean)."""
        n = int(nelem) * self.ctx.world_size
        if n != self._nelem:
            self._nelem = n
            self.ctx.nelem[self.slot] = float(n)

    @property
    def integer_bits(self):
        return int(self.ctx.exps[self.slot].item())

    def __repr__(self):
        return "Quantizer(%s, bits=%d, slot=%d)" % (self.name, self.bits, self.slot)


class DfxpContext:
    def __init__(self, device="cuda", capacity=1024, seed=0, world_size=1, sums_capacity=1 << 24):
        self.device = torch.device(device)
        self.capacity = capacity
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.world_size = int(world_size)
        dev = self.device
        self.exps = torch.zeros(capacity, dtype=torch.int32, device=dev)
        self.counts = torch.zeros(capacity * NSHARD * CSTRIDE, dtype=torch.int32, device=dev)
        self.step = torch.zeros(1, dtype=torch.int64, device=dev)
        self.bits = torch.zeros(capacity, dtype=torch.int32, device=dev)
        self.target = torch.zeros(capacity, dtype=torch.float32, device=dev)
        self.nelem = torch.zeros(capacity, dtype=torch.float32, device=dev)
        self.quantizers = []
        self.by_name = {}
        # per-step integer reduction buffers (BN channel sums, grad column sums), bump-allocated
        # from one arena so a whole step zeroes them with ONE fill (see zero_sums).
        self.sums_arena = torch.zeros(sums_capacity, dtype=torch.int64, device=dev)
        self._sums_used = 0
        self._extra_arenas = []
        self.sums_managed = False
        self.params_ready = False  # a model's batched prologue quantised every participating parameter  # True while a Trainer zeroes the arena once per step

    def quantizer(self, name, bits, initial=2, target=0.0, stochastic=True):
        """Register a quantiser (a ``*_range`` variable initialised to ``initial``)."""
        if name in self.by_name:
            raise ValueError("duplicate DFXP range variable %r" % name)
        if not 1 <= bits <= 32:  # weight_quantization's assertion (dynamic_fixed_point.py:21)
            raise ValueError("invalid value for bits: %d" % bits)
        if bits < 32 and not 0 <= bits - initial - 1 <= 30:
            raise ValueError("initial range %d invalid for %d bits (reference: 2**(bits-I-1) in int32)"
                             % (initial, bits))
        slot = len(self.quantizers)
        if slot >= self.capacity:
            raise RuntimeError("DfxpContext capacity exhausted")
        q = Quantizer(self, name, slot, bits, stochastic, target)
        self.exps[slot] = int(initial)
        self.bits[slot] = int(bits)
        self.target[slot] = float(target)
        self.quantizers.append(q)
        self.by_name[name] = q
        return q

    def noise_table_desc(self, q, inner):
        """A copy of stochastic quantiser q's descriptor whose noise comes from a per-step table of its
        `inner` noise values (u[i] for i < inner: the same Philox values the kernels draw inline,
        lbt_dfxp_noise_fill). For consumers that would otherwise recompute each value once per sample
        (the wide GEMMs' quantising epilogue: a tile's rows are pixels, the noise repeats over the
        batch). A new table is filled at once; fill_noise_tables (the model's per-step prologue)
        refills every table for the step that follows. A superseded table or job array is kept alive
        for the context's lifetime: a graph captured before may still launch the fill on it."""
        tabs = self.__dict__.setdefault("_ntab", {})
        ent = tabs.get(q.slot)
        if ent is None or ent[1] != inner:
            retired = self.__dict__.setdefault("_retired", [])
            if ent is not None:
                retired.append(ent)
            if getattr(self, "_njobs", None) is not None:
                retired.append(self._njobs)
            n4 = (int(inner) + 3) // 4 * 4
            tab = torch.empty(n4, dtype=torch.float32, device=self.device)
            d = QDesc.from_buffer_copy(q.desc)
            d.noise = tab.data_ptr()
            job = _lib.NJob(self.step.data_ptr(), self.seed, q.qid, 0, int(inner), tab.data_ptr())
            ent = (tab, int(inner), d, job)
            tabs[q.slot] = ent
            # job arrays uploaded here (eagerly: never inside a graph capture), the new table filled now
            self._njobs = self._job_array([e[3] for e in tabs.values()], max(e[1] for e in tabs.values()))
            dev, n, max_n = self._job_array([job], int(inner))
            retired.append(dev)  # read by the fill launched just below (stream-ordered, asynchronous)
            _lib.call("lbt_dfxp_noise_fill", _lib.ptr(dev), n, max_n, None, 0, _lib.stream())
        return ent[2]

    def _job_array(self, jobs, max_n):
        n = len(jobs)
        host = torch.frombuffer(bytearray(bytes((_lib.NJob * n)(*jobs))), dtype=torch.uint8)
        return host.to(self.device), n, int(max_n)

    def fill_noise_tables(self):
        """Refill every noise_table_desc table for the current step (one launch)."""
        if getattr(self, "_njobs", None) is None:
            return
        dev, n, max_n = self._njobs
        _lib.call("lbt_dfxp_noise_fill", _lib.ptr(dev), n, int(max_n), None, 0, _lib.stream())

    def alloc_sums(self, n):
        """n int64 from the arena. When the first arena is full (wide models: ResNet-50's weight-
        gradient slabs), further buffers come from overflow arenas of at least the same size --
        one more fill each per step."""
        n = (int(n) + 31) // 32 * 32
        if self._sums_used + n <= self.sums_arena.numel():
            t = self.sums_arena[self._sums_used:self._sums_used + n]
            self._sums_used += n
            return t
        for i, (arena, used) in enumerate(self._extra_arenas):
            if used + n <= arena.numel():
                self._extra_arenas[i] = (arena, used + n)
                return arena[used:used + n]
        arena = torch.zeros(max(n, self.sums_arena.numel()), dtype=torch.int64, device=self.device)
        self._extra_arenas.append((arena, n))
        return arena[:n]

    def zero_sums(self):
        if self._sums_used:
            self.sums_arena[: self._sums_used].zero_()
        for arena, used in self._extra_arenas:
            arena[:used].zero_()

    # the 'update_range' collection (trainer.py:63,157)
    def update_range_op(self, sgd=None):
        """The 'update_range' collection: one launch. sgd = (w, a, g, lr, mu, gscale) also runs the
        momentum optimiser in the same launch (lbt_step_update)."""
        n = len(self.quantizers)
        if sgd is None:
            _lib.call("lbt_dfxp_range_update", _lib.ptr(self.exps), _lib.ptr(self.counts), _lib.ptr(self.bits),
                      _lib.ptr(self.target), _lib.ptr(self.nelem), n, _lib.ptr(self.step), _lib.stream())
        else:
            w, a, g, lr, mu, gscale = sgd
            _lib.call("lbt_step_update", _lib.ptr(w), _lib.ptr(a), _lib.ptr(g), w.numel(), float(lr), float(mu),
                      float(gscale), _lib.ptr(self.exps), _lib.ptr(self.counts), _lib.ptr(self.bits),
                      _lib.ptr(self.target), _lib.ptr(self.nelem), n, _lib.ptr(self.step), _lib.stream())

    def update_range_folded_op(self, folded):
        """Data-parallel variant: the range update from all-reduced folded totals (see fold_counts)."""
        n = len(self.quantizers)
        _lib.call("lbt_dfxp_range_update_folded", _lib.ptr(self.exps), _lib.ptr(folded), _lib.ptr(self.bits),
                  _lib.ptr(self.target), _lib.ptr(self.nelem), n, _lib.ptr(self.step), _lib.stream())

    def fold_counts(self, folded):
        """Sum + zero every slot's counter shards into folded[4*slot ..] (exact fp32 hi/lo pairs)."""
        _lib.call("lbt_dfxp_counts_fold", _lib.ptr(self.counts), len(self.quantizers), _lib.ptr(folded),
                  _lib.stream())

    def counts_view(self):
        """[slots, NSHARD, 2] view of the live counters."""
        return self.counts.view(self.capacity, NSHARD, CSTRIDE)[: len(self.quantizers), :, :2]

    def ranges(self):
        """{range variable name: I} (host read -- not for the timed loop)."""
        e = self.exps[: len(self.quantizers)].cpu().tolist()
        return {q.name: int(v) for q, v in zip(self.quantizers, e)}

    def set_ranges(self, ranges):
        for name, v in ranges.items():
            self.exps[self.by_name[name].slot] = int(v)

    def state_dict(self):
        return {"exps": self.exps.clone(), "step": self.step.clone(),
                "names": [q.name for q in self.quantizers]}

    def load_state_dict(self, sd):
        names = [q.name for q in self.quantizers]
        if list(sd["names"]) != names:
            raise ValueError("quantiser layout mismatch")
        self.exps.copy_(sd["exps"])
        self.step.copy_(sd["step"])


_default = None


def default_context():
    """The process-wide context (the counterpart of TF's default graph)."""
    global _default
    if _default is None:
        _default = DfxpContext()
    return _default


def set_default_context(ctx):
    global _default
    _default = ctx
    return ctx
