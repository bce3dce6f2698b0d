"""Front end (wav -> FBANK -> sliding CMN) host logic: the FBANK oracle's
frame rule and filterbank, Kaldi config parsing, wav I/O, the FM ark writer
against the reference's kaldi_io bytes, and the C-ABI frame count.  The GPU
kernels are checked against the oracle in tests/test_frontend_gpu.py."""

import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_oracle_frame_rule():
    from oracle import fbank_ref
    # snip_edges: 1 + (N - 400) // 160, 0 below one window
    for n, t in ((0, 0), (399, 0), (400, 1), (559, 1), (560, 2), (16000, 98), (48017, 298)):
        assert fbank_ref.num_frames(n) == t


def test_oracle_mel_banks_shape_and_tone():
    from oracle import fbank_ref
    W = fbank_ref.mel_banks(80)
    assert W.shape == (80, 256)
    assert (W >= 0).all() and (W <= 1).all()
    assert (W.sum(1) > 0).all()                      # every bin has FFT bins
    assert W[:, 0].sum() == 0                        # DC (0 Hz) is below 20 Hz
    # a 1 kHz tone peaks in the mel bin whose center is nearest 1 kHz
    sr = 16000
    t = np.arange(sr) / sr
    x = (8000 * np.sin(2 * np.pi * 1000 * t)).astype(np.float32)
    f = fbank_ref.fbank(x, 80)
    mel = lambda hz: 1127 * np.log(1 + hz / 700)
    lo, hi = mel(20), mel(8000)
    centers = lo + (np.arange(80) + 1) * (hi - lo) / 81
    assert abs(int(np.median(f.argmax(1))) - int(np.abs(centers - mel(1000)).argmin())) <= 1


def test_oracle_silence_is_log_eps():
    from oracle import fbank_ref
    f = fbank_ref.fbank(np.zeros(1000, np.float32), 40)
    assert f.shape == (4, 40)
    assert np.all(f == np.float32(np.log(np.finfo(np.float32).eps)))


def test_config_parsing(tmp_path):
    from voxsrc2020_speaker_verification_amd.frontend import FbankOptions
    c = tmp_path / "fbank80.conf"
    c.write_text("--sample-frequency=16000\n--num-mel-bins=80\n")   # conf/fbank80.conf
    o = FbankOptions.from_config(str(c))
    assert (o.sample_frequency, o.num_mel_bins, o.dither, o.low_freq) == (16000.0, 80, 1.0, 20.0)
    c.write_text("--num-mel-bins=40\n--dither=0\n--preemphasis-coefficient=0.95\n")
    o = FbankOptions.from_config(str(c))
    assert (o.num_mel_bins, o.dither, o.preemphasis_coefficient) == (40, 0.0, 0.95)
    c.write_text("--window-type=hamming\n")
    with pytest.raises(ValueError):
        FbankOptions.from_config(str(c))


def test_wav_roundtrip(tmp_path):
    from voxsrc2020_speaker_verification_amd.frontend import read_wav, read_wav_scp, write_wav
    x = np.random.default_rng(0).integers(-32768, 32767, 1234).astype(np.float32)
    p = str(tmp_path / "a.wav")
    write_wav(p, x, 16000)
    y, rate = read_wav(p)
    assert rate == 16000 and y.dtype == np.float32 and np.array_equal(x, y)
    scp = tmp_path / "wav.scp"
    scp.write_text(f"utt1 {p}\n")
    assert read_wav_scp(str(scp)) == [("utt1", p)]
    scp.write_text("utt1 ffmpeg -i x.m4a -f wav - |\n")
    with pytest.raises(ValueError):
        read_wav_scp(str(scp))


def test_fm_writer_matches_kaldi_io_bytes():
    """format_mat_flt == kaldi_io.write_mat (golden fm_mats.ark)."""
    from voxsrc2020_speaker_verification_amd.kaldi import format_mat_flt
    exp = np.load(os.path.join(G, "fm_mats.npz"))
    raw = open(os.path.join(G, "fm_mats.ark"), "rb").read()
    got = b"".join(format_mat_flt(k, exp[k])[0] for k in ("m1", "m2"))
    assert got == raw
    rec, off = format_mat_flt("m1", exp["m1"])
    assert rec[off:off + 2] == b"\0B"


def test_abi_num_frames_matches_oracle():
    from oracle import fbank_ref
    from voxsrc2020_speaker_verification_amd import frontend
    o = frontend.FbankOptions(num_mel_bins=80)
    for n in (0, 399, 400, 560, 16000, 48017):
        assert frontend.num_frames(n, o) == fbank_ref.num_frames(n)
    o8 = frontend.FbankOptions(sample_frequency=8000, num_mel_bins=23)   # 200 / 80 samples
    assert frontend.num_frames(8000, o8) == 1 + (8000 - 200) // 80
