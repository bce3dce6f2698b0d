"""The C++/OpenMP fp32 CPU baseline (oracle/cpu/voxcpu.cpp: what bench.py's
cpu_baseline leg times, the stand-in for the reference's TF1 CPU `sess.run`)
computes the reference forward: within 1e-4 of the numpy fp32 oracle for every
backbone family."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def cpu():
    from oracle.cpu import build
    build.build()
    from oracle.cpu import CpuModel
    return CpuModel


@pytest.mark.parametrize("name,F,T,N", [("res2net50_w24_s4_c32", 80, 50, 2),
                                        ("res2net50_w24_s4_c32", 40, 37, 2),
                                        ("tdnn", 40, 120, 3), ("tdnn", 80, 200, 2),
                                        ("dpn68", 40, 33, 2),
                                        ("res2net101_w24_s4_c32_att", 16, 24, 2),
                                        ("res2net50_w8_s6_c16", 24, 40, 2)])
def test_cpu_baseline_matches_oracle(weights, cpu, name, F, T, N):
    from oracle import models_ref as R
    from voxsrc2020_speaker_verification_amd import synth
    spec, t, blob = weights(name, F)
    x = synth.make_features(N, T, F, seed=5) * np.float32(1.5)
    ref = R.forward(spec, t, x)
    m = cpu(blob)
    got = m.run(x, threads=4)
    assert got.shape == ref.shape
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err <= 1e-4, err
    # thread count does not change the result beyond float reassociation (none here)
    np.testing.assert_array_equal(m.run(x, threads=1), got)
