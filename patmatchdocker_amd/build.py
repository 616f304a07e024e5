"""Build the gfx950 HIP scan library in-tree (``libpatmatch_hip.so``).

``python -m patmatchdocker_amd.build`` cross-compiles every ``csrc/*.hip``
translation unit with hipcc (in parallel) and links them; no GPU is needed.
The .so is git-ignored but travels to the GPU box with the tree.
"""

from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libpatmatch_hip.so")
OBJDIR = os.path.join(HERE, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PM_OFFLOAD_ARCH", "gfx950")
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(ROOT, "include", "patmatch_hip.h")]


def _newer(target, deps):
    return os.path.exists(target) and all(os.path.getmtime(target) >= os.path.getmtime(d) for d in deps)


def _compile(src, verbose):
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    if _newer(obj, [src] + headers()):
        return obj
    cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    srcs = sources()
    if not force and _newer(OUT, srcs + headers()):
        return OUT
    os.makedirs(OBJDIR, exist_ok=True)
    if force:
        for f in glob.glob(os.path.join(OBJDIR, "*.o")):
            os.remove(f)
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), srcs))
    tmp = OUT + ".tmp"
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs + ["-lhiprtc"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
