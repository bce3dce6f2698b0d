"""The native reader (kaldi_host.cpp, host-only code) under AddressSanitizer and
UBSan: tools/asan/run.sh compiles it with g++ and a driver that walks the
golden FM / CM arks (every record whole and from every truncated prefix,
batched shape reads, ragged chunk reads with valid and invalid chunk tables,
through the worker pool and on the calling thread).  CPU only."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_reader_clean_under_asan_ubsan():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan", "run.sh")], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "ok (0 failures)" in r.stdout
