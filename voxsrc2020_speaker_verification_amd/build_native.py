"""Build libvoxemb.so in-tree with hipcc for gfx950 (no JIT cache: the .so
travels with the repo snapshot to the GPU box)."""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvoxemb.so")
# diagnostic build (-DVOX_DIAG: timing variants that skip work, for tools/;
# load it with VOXEMB_LIB=.../libvoxemb_diag.so)
DIAG_LIB = os.path.join(HERE, "libvoxemb_diag.so")
ARCH = os.environ.get("VOX_OFFLOAD_ARCH", "gfx950")

SOURCES = [
    ("kernels.hip", ["-O3"]),
    ("bneck.hip", ["-O3"]),
    ("asnorm.hip", ["-O3"]),
    ("gemm.hip", ["-O3"]),
    ("gemm_wide.hip", ["-O3"]),
    ("gconv.hip", ["-O3"]),
    ("conv3.hip", ["-O3"]),
    ("conv3r.hip", ["-O3"]),
    ("conv3k.hip", ["-O3"]),
    ("dpnblk.hip", ["-O3"]),
    ("conv3u.hip", ["-O3"]),
    ("conv3s.hip", ["-O3"]),
    ("gemm_nw.hip", ["-O3"]),
    ("fbank.hip", ["-O3"]),
    ("api.cpp", ["-O2"]),
    ("kaldi_host.cpp", ["-O2", "-ffp-contract=off", "--offload-host-only"]),
]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


# what the last build() call did: sources compiled, relinked, seconds
LAST_BUILD = {}


def build(verbose=False, force=False, diag=False) -> str:
    outdir = os.path.join(HERE, "..", "build", "native_diag" if diag else "native")
    lib = DIAG_LIB if diag else LIB
    dflags = ["-DVOX_DIAG"] if diag else []
    os.makedirs(outdir, exist_ok=True)
    hipcc = _hipcc()
    hdr = os.path.join(HERE, "..", "include", "voxemb.h")
    newest_hdr = max([os.path.getmtime(hdr), os.path.getmtime(__file__)] +
                     [os.path.getmtime(os.path.join(CSRC, n)) for n in os.listdir(CSRC)
                      if n.endswith(".h")])
    objs, relink, jobs = [], force or not os.path.exists(lib), []
    for src, flags in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(outdir, src + ".o")
        objs.append(obj)
        if (not force and os.path.exists(obj) and
                os.path.getmtime(obj) >= max(newest_hdr, os.path.getmtime(path))):
            continue
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        jobs.append([hipcc, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-c", *lang,
                     path, "-o", obj, *flags, *dflags])
    import time
    t0 = time.perf_counter()
    LAST_BUILD.clear()
    LAST_BUILD.update(compiled=[os.path.basename(j[j.index("-c") + (3 if j[j.index("-c") + 1] == "-x" else 1)])
                                for j in jobs], forced=bool(force), diag=bool(diag))
    if jobs:
        from concurrent.futures import ThreadPoolExecutor

        def _cc(cmd):
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)

        with ThreadPoolExecutor(max_workers=min(len(jobs), 6)) as pool:
            list(pool.map(_cc, jobs))
        relink = True
    if not relink and all(os.path.getmtime(lib) >= os.path.getmtime(o) for o in objs):
        LAST_BUILD.update(relinked=False, seconds=round(time.perf_counter() - t0, 1), lib=lib)
        return lib
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs]
    subprocess.run(cmd, check=True)
    LAST_BUILD.update(relinked=True, seconds=round(time.perf_counter() - t0, 1), lib=lib)
    return lib


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv, diag="--diag" in sys.argv))
