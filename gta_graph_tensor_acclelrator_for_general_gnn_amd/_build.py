"""Build libgta.so (hand-written HIP for gfx950) in-tree with hipcc.

No torch extension machinery: one hipcc invocation produces a plain C-ABI
shared library (include/gta.h) that any host language can bind.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "gta_kernels.hip")
OUT = os.path.join(HERE, "libgta.so")
ARCH = os.environ.get("GTA_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def needs_build(out=OUT):
    if not os.path.exists(out):
        return True
    deps = [SRC, os.path.join(HERE, "..", "include", "gta.h")]
    return any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
