"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every symbol the header
declares, and the ctypes structs match the C layouts (no GPU calls)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from lbt_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lbt_dfxp.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t)\s+(lbt_\w+)\s*\(", src, flags=re.M)))


def test_header_and_bindings_agree():
    assert header_functions() == _lib.EXPORTED


def test_library_loads_and_exports_every_symbol():
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.lbt_abi_version() == _lib.ABI_VERSION


def test_no_cpu_fallback_when_library_missing(tmp_path):
    with pytest.raises(ImportError):
        _lib.load.__wrapped__(str(tmp_path / "nope.so")) if hasattr(_lib.load, "__wrapped__") else \
            _load_fresh(str(tmp_path / "nope.so"))


def _load_fresh(path):
    saved = _lib._lib
    _lib._lib = None
    try:
        return _lib.load(path)
    finally:
        _lib._lib = saved


STRUCTS = {"lbt_qdesc": _lib.QDesc, "lbt_conv_desc": _lib.ConvDesc, "lbt_bn_norm": _lib.BnNorm,
           "lbt_chain_branch": _lib.ChainBranch, "lbt_chain_fwd": _lib.ChainFwd, "lbt_bwd_branch": _lib.BwdBranch,
           "lbt_chain_bwd_a": _lib.ChainBwdA, "lbt_chain_bwd_b": _lib.ChainBwdB, "lbt_wjob": _lib.WJob,
           "lbt_qjob": _lib.QJob, "lbt_rjob": _lib.RJob, "lbt_pjob": _lib.PJob, "lbt_r64job": _lib.R64Job, "lbt_njob": _lib.NJob,
           "lbt_head": _lib.Head, "lbt_xchg": _lib.Xchg, "lbt_fseg": _lib.FSeg,
           "lbt_wgrad_job": _lib.WgradJob, "lbt_conv_bwd": _lib.ConvBwd,
           "lbt_conv_fwd": _lib.ConvFwd, "lbt_conv_fwd_job": _lib.ConvFwdJob,
           "lbt_igemm_tuning": _lib.IgemmTuning, "lbt_update": _lib.Update,
           "lbt_dgrad_bna": _lib.DgradBna, "lbt_bna_bn": _lib.BnaBn, "lbt_dgrad_bn3": _lib.DgradBn3}


def test_struct_layouts_match_c():
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "lbt_dfxp.h"', 'int main(void){']
    for cname, py in STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write("\n".join(lines))
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        out = dict(l.rsplit(" ", 1) for l in subprocess.check_output([exe], text=True).splitlines())
    for cname, py in STRUCTS.items():
        assert int(out[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(out["%s.%s" % (cname, f)]) == getattr(py, f).offset, (cname, f)


def test_host_side_argument_checks_return_einval():
    """Entry points reject unsupported argument combinations on the host, before any HIP call (so this
    runs without a GPU): lbt_bn_chain_fwd's ReLU-mask bytes without the fp32 output they travel with,
    lbt_igemm_set_tuning's range checks (the accepted selection is restored), and the conv1 forward's
    fp16-exactness bound on the image codes."""
    lib = _lib.load()
    a = _lib.ChainFwd()
    a.rows, a.inner, a.C = 2, 64, 16
    a.ybits = ctypes.c_void_p(0x1000)  # never dereferenced: rejected first
    a.y = None
    assert lib.lbt_bn_chain_fwd(ctypes.byref(a), None) == 1001
    saved = _lib.IgemmTuning()
    assert lib.lbt_igemm_get_tuning(ctypes.byref(saved)) == 0
    assert saved.fwdq_perm == 2  # the default: staged, persistent for one-k-block forward GEMMs
    for field, bad in (("fwdq_perm", -1), ("stages", 5), ("max_bn", 96), ("min_tiles", 0)):
        t = _lib.IgemmTuning()
        ctypes.memmove(ctypes.byref(t), ctypes.byref(saved), ctypes.sizeof(t))
        setattr(t, field, bad)
        assert lib.lbt_igemm_set_tuning(ctypes.byref(t)) == 1001, field
    cur = _lib.IgemmTuning()
    lib.lbt_igemm_get_tuning(ctypes.byref(cur))
    assert (cur.fwdq_perm, cur.stages, cur.max_bn, cur.min_tiles) == \
        (saved.fwdq_perm, saved.stages, saved.max_bn, saved.min_tiles)
    # conv1 on fp16 MFMA: image codes wider than 12 bits are not exact in fp16 (|x| <= 2^11)
    d = _lib.ConvDesc(2, 224, 224, 3, 64, 7, 7, 2, 2, 3, 3, 3, 3, 112, 112)
    qx, qw = _lib.QDesc(), _lib.QDesc()
    qx.bits, qw.bits = 13, 2
    assert lib.lbt_conv_stem_wide_fwd(None, None, d, qx, qw, None, None) == 1001
