"""Build libvoxemb.so in-tree with hipcc for gfx950 (no JIT cache: the .so
travels with the repo snapshot to the GPU box)."""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvoxemb.so")
ARCH = os.environ.get("VOX_OFFLOAD_ARCH", "gfx950")

SOURCES = [
    ("kernels.hip", ["-O3"]),
    ("api.cpp", ["-O2"]),
    ("kaldi_host.cpp", ["-O2", "-ffp-contract=off"]),
]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def build(verbose=False, force=False) -> str:
    outdir = os.path.join(HERE, "..", "build", "native")
    os.makedirs(outdir, exist_ok=True)
    hipcc = _hipcc()
    objs = []
    newest_src = 0.0
    for name in os.listdir(CSRC):
        newest_src = max(newest_src, os.path.getmtime(os.path.join(CSRC, name)))
    hdr = os.path.join(HERE, "..", "include", "voxemb.h")
    newest_src = max(newest_src, os.path.getmtime(hdr), os.path.getmtime(__file__))
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= newest_src:
        return LIB
    for src, flags in SOURCES:
        obj = os.path.join(outdir, src + ".o")
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        cmd = [hipcc, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-c", *lang,
               os.path.join(CSRC, src), "-o", obj, *flags]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
    subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
