"""ORACLE (test infrastructure only) -- numpy restatement of Kaldi's
`compute-fbank-feats --config=conf/fbank80.conf` (prepare_data.sh:66-70; the
config sets only --sample-frequency=16000 --num-mel-bins=80, everything else is
Kaldi's default), the front end the reference runs before `copy-feats
--compress` and `apply-cmvn-sliding` (tf_extract.py:63).

Kaldi is not vendored in the reference and is absent here, so
this follows Kaldi's published algorithm (feature-window.cc ExtractWindow /
ProcessWindow, feature-fbank.cc FbankComputer::Compute, mel-computations.cc
MelBanks, feature-functions.cc ComputePowerSpectrum) with its defaults:
  * frames: 25 ms / 10 ms at 16 kHz (400 / 160 samples), snip_edges=true:
    n = 1 + (N - 400) // 160 frames (0 if N < 400);
  * per frame: [dither], DC removal (mean over the 400 samples), pre-emphasis
    0.97 (x[i] -= 0.97 x[i-1] for i = 399..1, x[0] -= 0.97 x[0]), "povey"
    window pow(0.5 - 0.5 cos(2 pi i / 399), 0.85), zero-padded to 512;
  * power spectrum |FFT|^2 of bins 0..256, mel filterbank of num_bins
    triangles between 20 Hz and Nyquist on mel(f) = 1127 ln(1 + f/700)
    (weights computed in float32 exactly as MelBanks does, FFT bins 0..255),
    log(max(energy, FLT_EPSILON)).
Differences from Kaldi that remain by construction: the FFT here is float64
(Kaldi: float32 split-radix), sums are in float64 (Kaldi: BLAS sdot), and
dither (Kaldi default 1.0, a random Gaussian per sample) is taken as 0 --
Kaldi's dithered features are not reproducible bit for bit by anyone.  So the
restatement is *parity unpinned* against Kaldi itself; it pins the GPU kernel
(csrc/fbank.hip) within a float32 tolerance.
"""

import numpy as np

F32 = np.float32
FLT_EPS = np.finfo(np.float32).eps


def num_frames(num_samples, frame_length=400, frame_shift=160):
    if num_samples < frame_length:
        return 0
    return 1 + (num_samples - frame_length) // frame_shift


def povey_window(frame_length=400):
    a = 2.0 * np.pi / (frame_length - 1)
    i = np.arange(frame_length, dtype=np.float64)
    return np.power(0.5 - 0.5 * np.cos(a * i), 0.85).astype(F32)


def mel_scale(f):
    f = np.asarray(f, F32)
    return (F32(1127.0) * np.log(F32(1.0) + f / F32(700.0))).astype(F32)


def mel_banks(num_bins=80, samp_freq=16000.0, padded=512, low_freq=20.0, high_freq=0.0):
    """MelBanks weights as a dense [num_bins, padded/2] float32 matrix."""
    num_fft_bins = padded // 2
    nyquist = F32(0.5 * samp_freq)
    high = F32(high_freq) if high_freq > 0 else F32(nyquist + F32(high_freq))
    fft_bin_width = F32(F32(samp_freq) / F32(padded))
    mel_low = mel_scale(F32(low_freq))
    mel_high = mel_scale(high)
    delta = F32((mel_high - mel_low) / F32(num_bins + 1))
    freqs = (fft_bin_width * np.arange(num_fft_bins, dtype=F32)).astype(F32)
    mels = mel_scale(freqs)
    W = np.zeros((num_bins, num_fft_bins), F32)
    for b in range(num_bins):
        left = F32(mel_low + F32(b) * delta)
        center = F32(mel_low + F32(b + 1) * delta)
        right = F32(mel_low + F32(b + 2) * delta)
        for i in range(num_fft_bins):
            m = mels[i]
            if left < m < right:
                if m <= center:
                    W[b, i] = F32((m - left) / (center - left))
                else:
                    W[b, i] = F32((right - m) / (right - center))
    return W


def fbank(wave, num_bins=80, samp_freq=16000.0, preemph=0.97, low_freq=20.0,
          high_freq=0.0, frame_length=400, frame_shift=160, padded=512):
    """[T, num_bins] float32 log-mel filterbank of a float waveform (int16
    sample values, as Kaldi reads them), dither 0."""
    wave = np.asarray(wave, F32)
    T = num_frames(wave.shape[0], frame_length, frame_shift)
    W = mel_banks(num_bins, samp_freq, padded, low_freq, high_freq).astype(np.float64)
    win = povey_window(frame_length).astype(np.float64)
    out = np.empty((T, num_bins), F32)
    for t in range(T):
        x = wave[t * frame_shift:t * frame_shift + frame_length].astype(np.float64)
        x = x - x.sum() / frame_length
        y = np.empty_like(x)
        y[1:] = x[1:] - preemph * x[:-1]
        y[0] = x[0] - preemph * x[0]
        y *= win
        buf = np.zeros(padded)
        buf[:frame_length] = y
        spec = np.fft.rfft(buf)
        power = spec.real ** 2 + spec.imag ** 2
        e = W @ power[:padded // 2]
        out[t] = np.log(np.maximum(e, FLT_EPS)).astype(F32)
    return out
