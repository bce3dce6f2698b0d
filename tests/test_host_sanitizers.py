"""Host AddressSanitizer/UBSan run of the native ark/scp reader (csrc/kaldi_host.cpp).

The reader parses untrusted Kaldi bytes (restating the reference's
kaldi_io.py:437-504 FM/CM decoders), so it is built here with
``-fsanitize=address,undefined -fno-sanitize-recover=all`` into a standalone
driver (tests/asan/kaldi_host_check.cpp) and run over the golden arks plus
deterministic mutations (bit flips, truncations, forged dimensions), every
file offset, sliding-CMN edge shapes and short FV-record buffers.  GPU
sanitizers are not available on the pool; this covers the host side.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(ROOT, "voxsrc2020_speaker_verification_amd", "csrc", "kaldi_host.cpp")
DRIVER = os.path.join(HERE, "asan", "kaldi_host_check.cpp")
GOLDEN = [os.path.join(HERE, "golden", f) for f in ("fm_mats.ark", "cm_mats.ark", "fv_records.ark")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not on PATH")
def test_kaldi_host_asan_ubsan(tmp_path):
    exe = str(tmp_path / "kaldi_host_check")
    cmd = ["g++", "-std=c++17", "-g", "-O1", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", SRC, DRIVER, "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "asan" in (b.stderr or "").lower():
        pytest.skip("ASan runtime unavailable: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe] + GOLDEN, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-3000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert lines[-1] == "ok"
    # the valid arks parse completely under both CM decoders
    counts = {l.split()[0].rsplit("/", 1)[-1] + l.split()[1]: int(l.split()[2].split("=")[1])
              for l in lines if "matrices=" in l}
    assert counts["fm_mats.arkkaldi=0"] == counts["fm_mats.arkkaldi=1"] > 0
    assert counts["cm_mats.arkkaldi=0"] == counts["cm_mats.arkkaldi=1"] > 0
