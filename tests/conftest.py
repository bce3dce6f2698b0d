import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: slower CPU test")


_WEIGHTS = {}


def weights_for(name, feat_dim, seed=1):
    """Synthetic calibrated weights (cached per session)."""
    key = (name, feat_dim, seed)
    if key not in _WEIGHTS:
        import io
        from voxsrc2020_speaker_verification_amd import archs, synth, weights
        spec = archs.get_arch(name, feat_dim)
        # Res2Nets: damped residual branches -> well-conditioned synthetic network,
        # so bf16-vs-fp32 checks are meaningful (synth.make_weights docstring)
        gain = 0.25 if spec["family"] == "res2net" else None
        t = synth.make_weights(spec, seed=seed, calib_n=8, calib_T=120, residual_gain=gain)
        buf = io.BytesIO()
        weights.save_blob(buf, spec, t)
        _WEIGHTS[key] = (spec, t, buf.getvalue())
    return _WEIGHTS[key]


@pytest.fixture
def weights():
    return weights_for
