"""Build an alternative copy of the library for A/B kernel studies (scratch builds).

    python tools/build_variant.py TAG [-DFLAG ...] [--src DIR]
    -> lbt_amd/build_var/TAG/liblbt_dfxp.so ; select it with LBT_LIBRARY=<path> (lbt_amd/_lib.py)

--src builds the .hip files of another directory (e.g. a `git worktree` of an older commit).
"""
import concurrent.futures
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
from lbt_amd import _build  # noqa: E402


def main():
    args = sys.argv[1:]
    tag = args.pop(0)
    src = None
    if "--src" in args:
        i = args.index("--src")
        src = args[i + 1]
        del args[i:i + 2]
    out = os.path.join(ROOT, "lbt_amd", "build_var", tag)
    os.makedirs(out, exist_ok=True)
    srcs = _build.sources() if src is None else sorted(
        os.path.join(src, f) for f in os.listdir(src) if f.endswith(".hip"))
    inc = [] if src is None else ["-I" + os.path.join(src, "..", "..", "include")]

    def one(s):
        obj = os.path.join(out, os.path.basename(s) + ".o")
        subprocess.check_call([_build.HIPCC] + inc + _build.FLAGS + args + ["-c", s, "-o", obj])
        return obj
    with concurrent.futures.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(one, srcs))
    lib = os.path.join(out, "liblbt_dfxp.so")
    subprocess.check_call([_build.HIPCC, "--offload-arch=" + _build.ARCH, "-shared", "-fPIC", "-o", lib] + objs)
    print(lib)


if __name__ == "__main__":
    main()
