"""Kaldi CompressedMatrix encoder (`copy-feats --compress=true`,
prepare_data.sh:69): the oracle restatement (oracle/kaldi_ref.cm_encode_kaldi)
against the native decoders.  Kaldi is absent, so the encoder is *parity
unpinned* against Kaldi itself; these CPU tests pin the oracle's internal
consistency (its payload decodes through vox_parse_mat_kaldi to exactly the
oracle's own CopyToMat restatement, within the codec's quantisation bound), and
tests/test_frontend_gpu.py holds vox_cm_compress_device to it byte for byte."""
import numpy as np
import pytest

from oracle import kaldi_ref as K
from voxsrc2020_speaker_verification_amd import kaldi


def _mats():
    rng = np.random.default_rng(5)
    yield (rng.standard_normal((300, 80)) * 4 + rng.standard_normal(80) * 6).astype(np.float32)
    yield (rng.standard_normal((9, 7))).astype(np.float32)            # smallest "CM "
    yield (rng.standard_normal((8, 5))).astype(np.float32)            # largest "CM2"
    yield (rng.standard_normal((1, 3))).astype(np.float32)
    q = np.round(rng.standard_normal((57, 11)) * 2).astype(np.float32)  # many ties
    q[:, 3] = 1.5                                                      # constant column
    yield q
    yield np.full((20, 4), -2.25, np.float32)                          # constant matrix


@pytest.mark.parametrize("i", range(6))
def test_cm_encode_decodes_natively(i):
    m = list(_mats())[i]
    tok, pl = K.cm_encode_kaldi(m)
    assert tok == (b"CM " if m.shape[0] > 8 else b"CM2 ")
    got, used = kaldi.parse_mat(b"\0B" + tok + pl, cm="kaldi")
    assert used == 2 + len(tok) + len(pl) and got.shape == m.shape
    ref = K.cm_decode_kaldi(pl) if tok == b"CM " else K.cm2_decode_kaldi(pl)
    assert np.array_equal(got, ref)
    # quantisation bound: the widest of the three piecewise-linear segments per
    # column (or one uint16 step for CM2) plus the header quantisation
    mn, rng = np.frombuffer(pl, np.float32, 2, 0)
    if tok == b"CM2 ":
        assert np.abs(got - m).max() <= rng / 65535 * 1.01
    else:
        cols = m.shape[1]
        h = np.frombuffer(pl, np.uint16, 4 * cols, 16).reshape(cols, 4).astype(np.float64)
        p = mn + rng * h / 65535.0
        step = np.maximum.reduce([(p[:, 1] - p[:, 0]) / 64, (p[:, 2] - p[:, 1]) / 128,
                                  (p[:, 3] - p[:, 2]) / 63])
        err = np.abs(got.astype(np.float64) - m).max(axis=0)
        assert np.all(err <= step / 2 + 2 * rng / 65535 + 1e-6 * (1 + np.abs(m).max()))


def test_cm2_rejected_by_kaldi_io_order():
    """kaldi_io's reader (kaldi_io.py:477) only accepts "CM "; so does ours in
    that mode, while cm="kaldi" reads CM2 as Kaldi C++ does."""
    tok, pl = K.cm_encode_kaldi(np.ones((3, 2), np.float32))
    assert tok == b"CM2 "
    with pytest.raises(Exception):
        kaldi.parse_mat(b"\0B" + tok + pl, cm="kaldi_io")
