"""Static check of the hand-counted vmcnt kernels (device_common.h): compile
each source with inline-asm vector-memory ops to gfx950 assembly (the product
flags).  A global load written as inline asm is invisible to the compiler's
waitcnt pass, which then believes its destination written at issue; the
register allocator may copy or reuse that register before the data lands.
That happened twice (the round-2 bneck_fused illegal-address fault, and again
in round 3 when compiling the diagnostic paths out changed the allocation), so
the row loads are now ordinary loads.  This test fails on the CPU, before any
GPU run, if an inline-asm load with a VGPR destination reappears in a kernel
whose simulated vector-memory queue (tools/vmcnt_audit.py, must-analysis over
the control-flow graph) shows an instruction touching a register such a load
will still write.  LDS-DMA loads (global_load_lds_*) have no VGPR destination."""
import os
import re
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "voxsrc2020_speaker_verification_amd", "csrc")
SOURCES = ["bneck.hip", "gemm.hip", "gemm_wide.hip", "conv3.hip", "conv3r.hip", "conv3s.hip",
           "conv3u.hip"]
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _hipcc():
    for c in ("/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    return None


ASM_LOAD = re.compile(r"^\s*(global|buffer|flat)_load_(?!lds)\w*\s+v")


def _asm_load_kernels(path):
    """kernels with an inline-asm (;;#ASMSTART .. ;;#ASMEND) load that has a
    VGPR destination"""
    out, name, inside = set(), None, False
    for line in open(path):
        if re.match(r"^_Z[\w.$]*:", line):
            name = line.split(":")[0]
        elif ";;#ASMSTART" in line:
            inside = True
        elif ";;#ASMEND" in line:
            inside = False
        elif inside and name and ASM_LOAD.match(line):
            out.add(name)
    return out


@pytest.mark.skipif(_hipcc() is None, reason="hipcc not available")
def test_no_inflight_register_hazards(tmp_path):
    import vmcnt_audit
    hipcc = _hipcc()

    def compile_one(src):
        out = str(tmp_path / (src + ".s"))
        cmd = [hipcc, "--offload-arch=gfx950", "-std=c++17", "-O3", "-x", "hip", "-S",
               "--cuda-device-only", os.path.join(CSRC, src), "-o", out]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-2000:]
        return out

    with ThreadPoolExecutor(max_workers=4) as pool:
        outs = list(pool.map(compile_one, SOURCES))
    bad, kernels = {}, 0
    for path in outs:
        asm_kernels = _asm_load_kernels(path)
        for name, ins in vmcnt_audit.parse(path).items():
            kernels += 1
            if name not in asm_kernels:
                continue   # every register-destination load is compiler-tracked
            hits, _ = vmcnt_audit.audit_must(ins)
            if hits:
                bad[name] = sorted({h[1] for h in hits})[:5]
    assert kernels >= 20
    assert not bad, bad
