"""Kaldi table I/O against the reference's kaldi_io (golden fixtures made by
tests/golden/make_golden.py) and sliding CMN against the oracle."""

import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_fv_records_bytes_match_kaldi_io():
    from voxsrc2020_speaker_verification_amd.kaldi import format_vec_flt
    ref = open(os.path.join(G, "fv_records.ark"), "rb").read()
    vec = np.load(os.path.join(G, "fv_records.npz"))
    keys = ["utt-a", "spk1-utt_2", "x", "empty"]
    got = b"".join(format_vec_flt(k, vec[k.replace("-", "_")])[0] for k in keys)
    assert got == ref


def test_read_vec_flt_ark_roundtrip():
    from voxsrc2020_speaker_verification_amd.kaldi import read_vec_flt_ark
    vec = np.load(os.path.join(G, "fv_records.npz"))
    got = dict(read_vec_flt_ark(os.path.join(G, "fv_records.ark")))
    assert list(got) == ["utt-a", "spk1-utt_2", "x", "empty"]
    for k, v in got.items():
        assert v.dtype == np.float32 and np.array_equal(v, vec[k.replace("-", "_")])


@pytest.mark.parametrize("name", ["fm_mats", "cm_mats"])
def test_read_mat_ark_bit_exact(name):
    """FM and CM (compressed) matrices decode bit-exactly as kaldi_io."""
    from voxsrc2020_speaker_verification_amd.kaldi import read_mat_ark
    exp = np.load(os.path.join(G, name + ".npz"))
    got = dict(read_mat_ark(os.path.join(G, name + ".ark")))
    assert sorted(got) == sorted(exp.files)
    for k in exp.files:
        assert got[k].shape == exp[k].shape
        assert np.array_equal(got[k].view(np.uint32), exp[k].astype(np.float32).view(np.uint32)), k


def test_read_mat_ark_cm_kaldi_cpp_order():
    """cm="kaldi": Kaldi C++ CompressedMatrix arithmetic (the values the
    reference's apply-cmvn-sliding pipe decodes), bit-exact vs the oracle's
    restatement; within a few float32 ULPs of kaldi_io's order."""
    from oracle import kaldi_ref
    from voxsrc2020_speaker_verification_amd.kaldi import read_mat_ark
    raw = open(os.path.join(G, "cm_mats.ark"), "rb").read()
    exp_io = np.load(os.path.join(G, "cm_mats.npz"))
    got = dict(read_mat_ark(os.path.join(G, "cm_mats.ark"), cm="kaldi"))
    assert sorted(got) == sorted(exp_io.files)
    ndiff = 0
    for k in exp_io.files:
        pos = raw.index(k.encode() + b" \0BCM ") + len(k) + 6
        ref = kaldi_ref.cm_decode_kaldi(raw[pos:])
        assert np.array_equal(got[k].view(np.uint32), ref.view(np.uint32)), k
        io = exp_io[k].astype(np.float32)
        np.testing.assert_allclose(got[k], io, rtol=4e-7, atol=4e-7 * np.abs(io).max())
        ndiff += int((got[k] != io).sum())
    # the two orders are genuinely different arithmetic on these fixtures
    assert ndiff > 0


def test_scp_offsets_and_ranges(tmp_path):
    """scp 'path:offset' lines point at '\\0B' (copy-vector ark,scp); matrix
    ranges [a:b,c:d] are inclusive as Kaldi's."""
    from voxsrc2020_speaker_verification_amd import kaldi
    ark = os.path.join(G, "fm_mats.ark")
    raw = open(ark, "rb").read()
    exp = np.load(os.path.join(G, "fm_mats.npz"))
    off_m2 = raw.index(b"m2 ") + 3
    m = kaldi.read_mat(ark, off_m2)
    assert np.array_equal(m, exp["m2"])
    scp = tmp_path / "f.scp"
    scp.write_text(f"a {ark}:{raw.index(b'm1 ') + 3}\nb {ark}:{off_m2}[2:5,0:9]\n")
    items = list(kaldi.iter_features(str(scp), cmn=False))
    assert [k for k, _ in items] == ["a", "b"]
    assert np.array_equal(items[1][1], exp["m2"][2:6, 0:10])
    # vector writer: ark bytes and scp offsets
    base = str(tmp_path / "xv")
    vecs = {"u1": np.arange(4, dtype=np.float32), "u2": -np.ones(3, np.float32)}
    with kaldi.VectorWriter(base) as w:
        for k, v in vecs.items():
            w.write(k, v)
    got = dict(kaldi.read_vec_flt_ark(base + ".ark"))
    assert all(np.array_equal(got[k], vecs[k]) for k in vecs)
    raw = open(base + ".ark", "rb").read()
    for line in open(base + ".scp"):
        key, rx = line.split()
        off = int(rx.rsplit(":", 1)[1])
        assert raw[off:off + 2] == b"\0B" and raw[off - len(key) - 1:off] == key.encode() + b" "


def test_truncated_and_unknown_matrices_fail():
    from voxsrc2020_speaker_verification_amd import _native, kaldi
    raw = open(os.path.join(G, "cm_mats.ark"), "rb").read()
    start = raw.index(b"\0B")
    with pytest.raises(_native.VoxError):
        kaldi.parse_mat(raw[start:start + 40])
    with pytest.raises(_native.VoxError):
        kaldi.parse_mat(b"\0BXM " + b"\0" * 20)
    with pytest.raises(_native.VoxError):
        kaldi.parse_mat(b" [ 1 2 ]\n")


@pytest.mark.parametrize("T", [1, 7, 150, 299, 300, 301, 451, 1200])
def test_sliding_cmn_matches_oracle(T):
    from oracle.kaldi_ref import sliding_cmn as ref
    from voxsrc2020_speaker_verification_amd.kaldi import sliding_cmn
    rng = np.random.default_rng(T)
    x = (rng.standard_normal((T, 23)) * 4 + 10).astype(np.float32)
    got = sliding_cmn(x)
    exp = ref(x)
    assert np.array_equal(got, exp)
    if T <= 300:  # whole-utterance mean subtraction
        np.testing.assert_allclose(got, x - x.astype(np.float64).mean(0), atol=1e-5)


def test_sliding_cmn_non_centered():
    from oracle.kaldi_ref import sliding_cmn as ref
    from voxsrc2020_speaker_verification_amd.kaldi import sliding_cmn
    x = np.random.default_rng(3).standard_normal((400, 5)).astype(np.float32)
    assert np.array_equal(sliding_cmn(x, 300, center=False), ref(x, 300, center=False))


def test_write_many_bytes_equal_per_record_writer(tmp_path):
    """VectorWriter.write_many (the merged-ark writer of dp_extract) writes the
    same ark and scp bytes as one write() per vector (vox_format_vec_flt, whose
    records equal kaldi_io.write_vec_flt's, golden above)."""
    from voxsrc2020_speaker_verification_amd.kaldi import VectorWriter
    rng = np.random.default_rng(3)
    keys = [f"id{i:05d}-utt_{i * 7}" for i in range(37)] + ["x"]
    emb = rng.standard_normal((len(keys), 256)).astype(np.float32)
    with VectorWriter(str(tmp_path / "a")) as w:
        for k, v in zip(keys, emb):
            w.write(k, v)
    with VectorWriter(str(tmp_path / "b")) as w:
        w.write("first", emb[0])               # offsets continue after earlier records
        w.write_many(keys, emb)
    with VectorWriter(str(tmp_path / "c")) as w:
        w.write("first", emb[0])
        for k, v in zip(keys, emb):
            w.write(k, v)
    assert (tmp_path / "b.ark").read_bytes() == (tmp_path / "c.ark").read_bytes()
    assert ((tmp_path / "b.scp").read_text().replace("/b.ark", "/c.ark")
            == (tmp_path / "c.scp").read_text())
    with VectorWriter(str(tmp_path / "d")) as w:
        w.write_many(keys, emb)
    assert (tmp_path / "d.ark").read_bytes() == (tmp_path / "a.ark").read_bytes()
    with pytest.raises(ValueError):
        with VectorWriter(str(tmp_path / "e")) as w:
            w.write_many(["bad key"], emb[:1])
