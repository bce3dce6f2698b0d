"""wav -> FBANK -> sliding CMN on the device: the front half of the reference
pipeline, so wav -> embedding runs entirely on the GPU.

Reference steps replaced:
  * `compute-fbank-feats --config=conf/fbank80.conf scp:wav.scp ark:-`
    (prepare_data.sh:66-70; Kaldi feature-fbank.cc, not vendored) -> `fbank`
    / the `compute-fbank-feats`-style CLI below (FM ark + scp out);
  * `apply-cmvn-sliding --norm-vars=false --center=true --cmn-window=300`
    (tensorflow/tf_extract.py:63) -> `sliding_cmn` (bit-identical to the host
    `kaldi.sliding_cmn`);
  * `tf_extract.py` on those features -> `embed_wavs` (chunk rule and
    batching of `extract.embed_utterances`, features never leave HBM).
  * `copy-feats --compress=true` (prepare_data.sh:69) between the two Kaldi
    steps -> `cm_compress_device` (Kaldi CompressedMatrix, kAutomaticMethod):
    the lossy 8-bit codec the reference's features pass through.  Opt-in
    (`embed_wavs(compress=True)`, CLI `--compress`), so reference-parity runs
    see the same quantised features; `kaldi.read_mat(..., cm="kaldi")`
    decodes the written arks exactly as Kaldi does.
Kaldi's default dither (1.0, random) is supported with a counter-based
generator keyed by (seed, utterance key, frame, sample): each utterance draws
its own noise, as Kaldi's per-utterance RandomState does, and the result does
not depend on batch composition; dither=0 gives deterministic features (used by
the parity tests).

Kernels: libvoxemb `vox_fbank_device_keyed` / `vox_cm_compress_device` /
`vox_sliding_cmn_device` (csrc/fbank.hip).  No CPU fallback.

    python -m voxsrc2020_speaker_verification_amd.frontend \\
        --config conf/fbank80.conf scp:data/voxceleb1/wav.scp \\
        ark,scp:data/voxceleb1/fbank80.ark,data/voxceleb1/fbank80.scp
"""

from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import os
import struct
import sys
from dataclasses import dataclass, fields

import numpy as np

from ._native import FbankOpts, check, lib


@dataclass
class FbankOptions:
    """Kaldi FbankOptions / FrameExtractionOptions / MelBanksOptions subset
    (defaults are Kaldi's, except num_mel_bins 80 as conf/fbank80.conf)."""
    sample_frequency: float = 16000.0
    frame_length_ms: float = 25.0
    frame_shift_ms: float = 10.0
    dither: float = 1.0
    preemphasis_coefficient: float = 0.97
    remove_dc_offset: bool = True
    num_mel_bins: int = 80
    low_freq: float = 20.0
    high_freq: float = 0.0
    seed: int = 0

    def c(self):
        o = FbankOpts()
        for f in fields(self):
            setattr(o, f.name, int(getattr(self, f.name)) if f.name in
                    ("remove_dc_offset", "num_mel_bins", "seed") else float(getattr(self, f.name)))
        return o

    @classmethod
    def from_config(cls, path, **over):
        """Parse a Kaldi config file (`--sample-frequency=16000` lines)."""
        o = cls()
        names = {f.name.replace("_", "-"): f.name for f in fields(cls)}
        names["preemphasis-coefficient"] = "preemphasis_coefficient"
        with open(path) as fh:
            for line in fh:
                line = line.split("#", 1)[0].strip()
                if not line:
                    continue
                if not line.startswith("--") or "=" not in line:
                    raise ValueError(f"{path}: cannot parse {line!r}")
                k, v = line[2:].split("=", 1)
                if k not in names:
                    raise ValueError(f"{path}: option --{k} is not supported")
                setattr(o, names[k], _coerce(getattr(o, names[k]), v))
        for k, v in over.items():
            setattr(o, k, v)
        return o


def _coerce(cur, v):
    if isinstance(cur, bool):
        return v.lower() in ("1", "true")
    return type(cur)(v)


def num_frames(num_samples, opts=None):
    opts = opts or FbankOptions()
    return check(lib().vox_fbank_num_frames(int(num_samples), C.byref(opts.c())))


# ------------------------------------------------------------------ wav I/O
def read_wav(path):
    """RIFF/WAVE PCM16 mono (or the first channel) -> float32 sample values,
    as Kaldi's WaveData reads them (not normalised), and the sample rate."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, ch, rate, _, _, bits = fmt
    if tag != 1 or bits != 16:
        raise ValueError(f"{path}: only 16-bit PCM is supported (tag {tag}, {bits} bits)")
    x = np.frombuffer(pcm[:len(pcm) // (2 * ch) * 2 * ch], "<i2").reshape(-1, ch)[:, 0]
    return x.astype(np.float32), rate


def write_wav(path, samples, rate=16000):
    x = np.clip(np.round(np.asarray(samples, np.float64)), -32768, 32767).astype("<i2")
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 36 + 2 * x.size) + b"WAVE")
        f.write(b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, rate, 2 * rate, 2, 16))
        f.write(b"data" + struct.pack("<I", 2 * x.size) + x.tobytes())


def read_wav_scp(path):
    """`key path` lines (the reference's wav.scp entries are ffmpeg/sox pipes,
    prepare_data.sh:40-52; decode those to .wav first)."""
    out = []
    with open(path) as f:
        for line in f:
            t = line.strip().split(None, 1)
            if not t:
                continue
            if len(t) < 2 or t[1].rstrip().endswith("|"):
                raise ValueError(f"{path}: only plain wav paths are supported: {line.strip()!r}")
            out.append((t[0], t[1].strip()))
    return out


# ------------------------------------------------------------------ device ops
def utt_dither_key(key):
    """64-bit dither key of an utterance id (stable across runs and hosts)."""
    return int.from_bytes(hashlib.blake2b(str(key).encode(), digest_size=8).digest(), "little")


def _dev(device):
    import torch
    return torch.device("cuda", device) if isinstance(device, int) else torch.device(device)


def fbank_device(waves, opts=None, device=0, stream=None, keys=None):
    """waves: list of 1-D float arrays/tensors; keys: optional utterance ids
    (one per wave) that key the dither noise per utterance.  Returns (feats
    [sum T, bins] float32 on the device, frame offsets int64 [n+1] host)."""
    import torch
    opts = opts or FbankOptions()
    dev = _dev(device)
    lens = [int(w.shape[0]) for w in waves]
    samp_off = np.zeros(len(waves) + 1, np.int64)
    samp_off[1:] = np.cumsum(lens)
    frames = [num_frames(n, opts) for n in lens]
    frame_off = np.zeros(len(waves) + 1, np.int64)
    frame_off[1:] = np.cumsum(frames)
    with torch.cuda.device(dev):
        flat = torch.empty(int(samp_off[-1]), dtype=torch.float32, device=dev)
        for w, a in zip(waves, samp_off[:-1]):
            t = w if isinstance(w, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(w, np.float32))
            flat[int(a):int(a) + t.shape[0]] = t.to(dev, torch.float32)
        so = torch.from_numpy(samp_off).to(dev)
        fo = torch.from_numpy(frame_off).to(dev)
        uk = None
        if keys is not None:
            if len(keys) != len(waves):
                raise ValueError(f"{len(keys)} keys for {len(waves)} waveforms")
            kv = np.array([utt_dither_key(k) for k in keys], np.uint64).view(np.int64)
            uk = torch.from_numpy(kv).to(dev)
        out = torch.empty((int(frame_off[-1]), opts.num_mel_bins), dtype=torch.float32, device=dev)
        s = stream or torch.cuda.current_stream(dev)
        # the uploads above ran on the current stream: order the kernel after them
        s.wait_stream(torch.cuda.current_stream(dev))
        if len(waves):
            check(lib().vox_fbank_device_keyed(
                C.c_void_p(flat.data_ptr()), C.c_void_p(so.data_ptr()), C.c_void_p(fo.data_ptr()),
                C.c_void_p(uk.data_ptr() if uk is not None else None), len(waves),
                int(frame_off[-1]), C.byref(opts.c()), C.c_void_p(out.data_ptr()),
                C.c_void_p(s.cuda_stream)))
        s.synchronize()   # the offsets / waveform tensors die with this frame
    return out, frame_off


def sliding_cmn_device(feats, frame_off, cmn_window=300, center=True, stream=None):
    """Kaldi apply-cmvn-sliding over every utterance of a concatenated device
    feature matrix (frame offsets frame_off [n+1])."""
    import torch
    dev = feats.device
    n = len(frame_off) - 1
    out = torch.empty_like(feats)
    if n <= 0 or feats.shape[0] == 0:
        return out
    with torch.cuda.device(dev):
        fo = torch.from_numpy(np.asarray(frame_off, np.int64)).to(dev)
        s = stream or torch.cuda.current_stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))   # fo and feats were produced there
        check(lib().vox_sliding_cmn_device(C.c_void_p(feats.data_ptr()), C.c_void_p(fo.data_ptr()),
                                           n, feats.shape[1], int(cmn_window), 1 if center else 0,
                                           C.c_void_p(out.data_ptr()), C.c_void_p(s.cuda_stream)))
        s.synchronize()
    return out


def cm_blob_bytes(rows, cols):
    """Bytes of a compressed payload after its "CM " (rows > 8) / "CM2 " token."""
    return check(lib().vox_cm_blob_bytes(int(rows), int(cols)))


def cm_compress_device(feats, frame_off, stream=None, decode=True):
    """`copy-feats --compress=true` over every utterance of a concatenated
    device feature matrix: returns (decoded features [sum T, F] float32 on the
    device as Kaldi's CopyToMat yields them, or None; uint8 device blob; int64
    host blob offsets [n+1]).  Utterance u's payload is
    blob[off[u]:off[u+1]], to follow b"CM " if it has > 8 frames else b"CM2 " (Kaldi tokens end in a space)."""
    import torch
    dev = feats.device
    fo = np.asarray(frame_off, np.int64)
    n, F = len(fo) - 1, int(feats.shape[1])
    sizes = [cm_blob_bytes(int(fo[i + 1] - fo[i]), F) for i in range(n)]
    boff = np.zeros(n + 1, np.int64)
    boff[1:] = np.cumsum(sizes)
    blob = torch.empty(int(boff[-1]), dtype=torch.uint8, device=dev)
    out = torch.empty_like(feats) if decode else None
    if n <= 0:
        return out, blob, boff
    with torch.cuda.device(dev):
        fo_d = torch.from_numpy(fo).to(dev)
        bo_d = torch.from_numpy(boff[:-1].copy()).to(dev)
        s = stream or torch.cuda.current_stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        for lo in range(0, n, 65535):    # grid.y limit
            hi = min(n, lo + 65535)
            check(lib().vox_cm_compress_device(
                C.c_void_p(feats.data_ptr()), C.c_void_p(fo_d[lo:].data_ptr()), hi - lo, F,
                C.c_void_p(blob.data_ptr()), C.c_void_p(bo_d[lo:].data_ptr()),
                C.c_void_p(out.data_ptr() if out is not None else None),
                C.c_void_p(s.cuda_stream)))
        s.synchronize()
    return out, blob, boff


def format_cm_record(key, payload, rows):
    """Bytes of one compressed ark record and the offset of its '\\0B'."""
    k = key.encode("utf-8")
    if not k or b" " in k:
        raise ValueError("key must be non-empty without spaces")
    # Kaldi WriteToken appends a space: "CM" -> b"CM ", "CM2" -> b"CM2 "
    return k + b" \0B" + (b"CM " if rows > 8 else b"CM2 ") + bytes(payload), len(k) + 1


def fbank(waves, opts=None, device=0, cmn=False, keys=None):
    """Host convenience: list of waveforms -> list of [T, bins] numpy arrays."""
    feats, fo = fbank_device(waves, opts, device, keys=keys)
    if cmn:
        feats = sliding_cmn_device(feats, fo)
    h = feats.cpu().numpy()
    return [h[fo[i]:fo[i + 1]] for i in range(len(waves))]


def embed_wavs(extractor, waves, opts=None, batch=64, cmn=True, keys=None, compress=False):
    """wav -> embeddings with features resident on the device: fbank,
    [CM round trip,] CMN, the tf_extract chunk rule (<= 1000-frame chunks,
    length-weighted mean) with equal-length chunks batched
    (extract.embed_utterances).  keys: utterance ids for the per-utterance
    dither stream; compress: apply the reference's `copy-feats --compress`
    quantisation (prepare_data.sh:69) before CMN."""
    import torch
    from .extract import embed_utterances
    feats, fo = fbank_device(waves, opts, extractor.device, keys=keys)
    if compress:
        feats, _, _ = cm_compress_device(feats, fo)
    if cmn:
        feats = sliding_cmn_device(feats, fo)
    dev = feats.device
    utts = [(str(i), feats[fo[i]:fo[i + 1]]) for i in range(len(waves))]

    def embed_batch(x):   # x: stacked device chunks [n, L, F]
        # staged buffers per shape: same-shape batches replay one captured graph
        out = extractor.run_device_staged(x)
        torch.cuda.synchronize(dev)
        return out.cpu().numpy()

    return embed_utterances(utts, embed_batch, extractor.dim, batch, stack=torch.stack)


# ------------------------------------------------------------------ CLI
def _parse_wspec(spec):
    if spec.startswith("ark,scp:"):
        a, s = spec[len("ark,scp:"):].split(",")
        return a, s
    if spec.startswith("ark:"):
        return spec[4:], None
    raise ValueError(f"unsupported wspecifier {spec!r} (ark:<file> or ark,scp:<ark>,<scp>)")


def main(argv=None):
    ap = argparse.ArgumentParser(description="compute-fbank-feats on the GPU")
    ap.add_argument("--config", default=None, help="Kaldi config (conf/fbank80.conf)")
    ap.add_argument("--dither", type=float, default=None)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--batch", type=int, default=256, help="utterances per device call")
    ap.add_argument("--compress", default="false", choices=["true", "false"],
                    help="write Kaldi compressed (CM) matrices, as copy-feats --compress=true")
    ap.add_argument("rspec", help="scp:wav.scp")
    ap.add_argument("wspec", help="ark:feats.ark or ark,scp:feats.ark,feats.scp")
    a = ap.parse_args(argv)
    opts = FbankOptions.from_config(a.config) if a.config else FbankOptions()
    if a.dither is not None:
        opts.dither = a.dither
    if not a.rspec.startswith("scp:"):
        raise SystemExit("rspecifier must be scp:<wav.scp>")
    items = read_wav_scp(a.rspec[4:])
    ark, scp = _parse_wspec(a.wspec)
    from .kaldi import format_mat_flt
    with open(ark, "wb") as fa, (open(scp, "w") if scp else open(os.devnull, "w")) as fs:
        for b in range(0, len(items), a.batch):
            part = items[b:b + a.batch]
            waves = []
            for key, path in part:
                w, rate = read_wav(path)
                if rate != int(opts.sample_frequency):
                    raise SystemExit(f"{key}: sample rate {rate} != {opts.sample_frequency}")
                waves.append(w)
            keys = [k for k, _ in part]
            if a.compress == "true":
                feats, fo = fbank_device(waves, opts, a.device, keys=keys)
                _, blob, boff = cm_compress_device(feats, fo, decode=False)
                hb = blob.cpu().numpy()
                recs = [format_cm_record(k, hb[boff[i]:boff[i + 1]], int(fo[i + 1] - fo[i]))
                        for i, k in enumerate(keys)]
            else:
                recs = [format_mat_flt(k, m) for k, m in zip(keys, fbank(waves, opts, a.device,
                                                                         keys=keys))]
            for key, (rec, off) in zip(keys, recs):
                pos = fa.tell()
                fa.write(rec)
                fs.write(f"{key} {ark}:{pos + off}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
