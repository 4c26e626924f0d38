"""Build libgta.so (hand-written HIP for gfx950) in-tree with hipcc.

No torch extension machinery: one hipcc invocation produces a plain C-ABI
shared library (include/gta.h) that any host language can bind.
"""
import hashlib
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


HDR = os.path.join(HERE, "..", "include", "gta.h")


def source_id(paths=None):
    """First 16 hex digits of sha256 over the kernel source and the ABI header, the id compiled
    into libgta.so as gta_build_id(); None if a source is missing."""
    h = hashlib.sha256()
    for p in paths or (SRC, HDR):
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def needs_build(out=OUT):
    if not os.path.exists(out):
        return True
    return any(os.path.getmtime(d) > os.path.getmtime(out) for d in (SRC, HDR))


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           f'-DGTA_BUILD_ID="{source_id()}"', "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    # every in-flight load covered before its registers are touched (inline-asm loads included)
    from . import asmcheck
    hazards, n = asmcheck.check_library(OUT + ".tmp")
    if hazards:
        for h in hazards[:20]:
            print("asmcheck hazard:", h, file=sys.stderr)
        os.replace(OUT + ".tmp", OUT + ".rejected")  # kept for inspection (python -m ...asmcheck libgta.so.rejected)
        raise RuntimeError(f"asmcheck: {len(hazards)} register hazards in the built code object; libgta.so not "
                           f"installed (the binary is left at {OUT}.rejected)")
    if verbose:
        print(f"asmcheck: {n} kernels, no register touched while its load is in flight", flush=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
