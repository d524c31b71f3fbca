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
           "lbt_qjob": _lib.QJob, "lbt_rjob": _lib.RJob, "lbt_pjob": _lib.PJob, "lbt_njob": _lib.NJob,
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
