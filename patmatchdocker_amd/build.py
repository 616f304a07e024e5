"""Build the gfx950 HIP scan library in-tree (``libpatmatch_hip.so``).

``python -m patmatchdocker_amd.build`` cross-compiles with hipcc; no GPU is
needed.  The .so is git-ignored but travels to the GPU box with the tree.
"""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "pm_scan.hip")
OUT = os.path.join(HERE, "libpatmatch_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PM_OFFLOAD_ARCH", "gfx950")


def command(out: str = OUT):
    return [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
            "-I" + os.path.join(ROOT, "include"), "-o", out, SRC, "-lhiprtc"]


def build(force: bool = False, verbose: bool = False) -> str:
    deps = [SRC, os.path.join(ROOT, "include", "patmatch_hip.h")]
    if not force and os.path.exists(OUT) and \
            all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    cmd = command()
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    tmp = OUT + ".tmp"
    subprocess.run(cmd[:-4] + ["-o", tmp, SRC, "-lhiprtc"], check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
