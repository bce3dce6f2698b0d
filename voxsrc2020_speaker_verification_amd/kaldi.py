"""Kaldi table I/O for the extraction path, without Kaldi binaries.

Replaces, for this path:
  * the rspec pipe `ark:apply-cmvn-sliding --norm-vars=false --center=true
    --cmn-window=300 scp:<rspec>.scp ark:- |` (tensorflow/tf_extract.py:63) ->
    `iter_features(scp)`: scp parse, binary matrix read (FM/DM/CM), sliding CMN
    (native, libvoxemb);
  * the wspec pipe `ark:| copy-vector ark:- ark,scp:<wspec>.ark,<wspec>.scp`
    (tf_extract.py:65) + kaldi_io.write_vec_flt (kaldi_io.py:304-334) ->
    `VectorWriter`: FV records byte-identical to kaldi_io, plus the scp;
  * kaldi_io.read_vec_flt_ark (kaldi_io.py:249-300) -> `read_vec_flt_ark`.
"""

from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

from ._native import check, fptr, lib

CMN_WINDOW = 300


def read_scp(path):
    """[(key, rxfile)] from a Kaldi scp (`key rxfile` per line)."""
    out = []
    with open(path, "r") as f:
        for ln in f:
            ln = ln.strip()
            if not ln:
                continue
            key, rx = ln.split(None, 1)
            out.append((key, rx))
    return out


_RANGE = re.compile(r"^(.+)\[(.+)\]$")


def parse_rxfile(rx):
    """'path:offset[range]' -> (path, offset, (row_slice, col_slice) or None)."""
    rng = None
    m = _RANGE.match(rx)
    if m:
        rx, r = m.group(1), m.group(2)
        sl = []
        for part in r.split(","):
            a, b = part.split(":")
            sl.append(slice(int(a) if a else None, int(b) + 1 if b else None))
        rng = tuple(sl)
    mo = re.search(r":([0-9]+)$", rx)
    if mo:
        return rx[:mo.start()], int(mo.group(1)), rng
    return rx, 0, rng


CM_DECODE = ("kaldi_io", "kaldi")


def _cm_fn(cm, name):
    if cm not in CM_DECODE:
        raise ValueError(f"cm must be one of {CM_DECODE}")
    return getattr(lib(), name + ("_kaldi" if cm == "kaldi" else ""))


def read_mat(path, offset=0, cm="kaldi_io"):
    """Binary Kaldi matrix (FM / DM / CM) at `offset` -> float32 [rows, cols].
    cm="kaldi_io": compressed payloads decoded in kaldi_io._read_compressed_mat's
    arithmetic (the reference's Python reader); cm="kaldi": in Kaldi C++'s
    CompressedMatrix arithmetic (what the reference's apply-cmvn-sliding pipe
    decodes, tf_extract.py:63)."""
    r, c = C.c_int(), C.c_int()
    check(lib().vox_mat_shape(os.fsencode(path), int(offset), C.byref(r), C.byref(c)))
    out = np.empty((r.value, c.value), np.float32)
    check(_cm_fn(cm, "vox_read_mat")(os.fsencode(path), int(offset), fptr(out), r.value,
                                     c.value))
    return out


def parse_mat(buf, cm="kaldi_io"):
    """Binary matrix from bytes starting at '\\0B' -> (float32 array, bytes used)."""
    r, c = C.c_int(), C.c_int()
    check(lib().vox_parse_mat_shape(buf, len(buf), C.byref(r), C.byref(c)))
    out = np.empty((r.value, c.value), np.float32)
    used = C.c_size_t()
    check(_cm_fn(cm, "vox_parse_mat")(buf, len(buf), fptr(out), r.value, c.value,
                                      C.byref(used)))
    return out, used.value


def _read_key(buf, pos):
    end = buf.index(b" ", pos)
    return buf[pos:end].decode("utf-8").strip(), end + 1


def read_mat_ark(path, cm="kaldi_io"):
    """Generator of (key, matrix) over an ark of binary matrices (kaldi_io.read_mat_ark)."""
    with open(path, "rb") as f:
        buf = f.read()
    pos = 0
    while pos < len(buf):
        key, pos = _read_key(buf, pos)
        if not key:
            break
        mat, used = parse_mat(buf[pos:], cm)
        pos += used
        yield key, mat


def sliding_cmn(x, cmn_window=CMN_WINDOW, center=True):
    """Kaldi apply-cmvn-sliding --norm-vars=false (double-precision running sums)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    T, F = x.shape
    check(lib().vox_sliding_cmn(fptr(x), T, F, int(cmn_window), 1 if center else 0, fptr(out)))
    return out


def iter_features(scp_path, cmn=True, cm="kaldi"):
    """(key, float32 [T, F]) in scp order: the tf_extract rspec pipeline
    (Kaldi decodes compressed arks there, hence cm="kaldi")."""
    for key, rx in read_scp(scp_path):
        path, off, rng = parse_rxfile(rx)
        mat = read_mat(path, off, cm)
        if rng is not None:
            mat = np.ascontiguousarray(mat[rng])
        yield key, (sliding_cmn(mat) if cmn else mat)


def format_vec_flt(key, v):
    """Bytes of one FV ark record and the offset of its '\\0B' (for the scp)."""
    v = np.ascontiguousarray(v, dtype=np.float32)
    off = C.c_int64()
    k = key.encode("utf-8")
    need = lib().vox_format_vec_flt(k, fptr(v), v.shape[0], None, 0, C.byref(off))
    check(need)
    buf = C.create_string_buffer(need)
    check(lib().vox_format_vec_flt(k, fptr(v), v.shape[0], buf, need, C.byref(off)))
    return buf.raw[:need], off.value


def format_mat_flt(key, m):
    """Bytes of one binary FM ark record ("key \\0BFM \\4<i32 rows>\\4<i32 cols>
    <f32 data>", kaldi_io.write_mat's layout, kaldi_io.py:508-540) and the
    offset of its '\\0B' (for the scp)."""
    m = np.ascontiguousarray(m, dtype=np.float32)
    if m.ndim != 2:
        raise ValueError("expected a 2-D matrix")
    k = key.encode("utf-8")
    if not k or b" " in k:
        raise ValueError("key must be non-empty without spaces")
    head = k + b" \0BFM \4" + np.int32(m.shape[0]).tobytes() + b"\4" + np.int32(m.shape[1]).tobytes()
    return head + m.tobytes(), len(k) + 1


class VectorWriter:
    """`ark,scp:<base>.ark,<base>.scp` writer of float vectors (copy-vector)."""

    def __init__(self, base, atomic=False):
        """atomic=True: write <base>.ark/.scp under temporary names and rename
        them into place on close (ark first, then scp), so an interrupted
        writer never leaves a complete-looking pair (dp_extract --resume)."""
        self.ark_path = base + ".ark"
        self.scp_path = base + ".scp"
        self._atomic = atomic
        sfx = f".part{os.getpid()}" if atomic else ""
        self._ark = open(self.ark_path + sfx, "wb")
        self._scp = open(self.scp_path + sfx, "w")
        self._sfx = sfx

    def write(self, key, v):
        rec, off = format_vec_flt(key, v)
        pos = self._ark.tell()
        self._ark.write(rec)
        self._scp.write(f"{key} {self.ark_path}:{pos + off}\n")

    def write_many(self, keys, emb):
        """write() for every (key, row) of a [n, dim] matrix: the same bytes as
        vox_format_vec_flt per record, assembled here in one pass (a 1.09 M
        utterance merged ark is ~1 s instead of one native call per vector)."""
        emb = np.ascontiguousarray(emb, dtype=np.float32)
        if emb.ndim != 2 or len(keys) != emb.shape[0]:
            raise ValueError("expected one key per row of a 2-D matrix")
        mid = np.frombuffer(b" \0BFV \4" + np.uint32(emb.shape[1]).tobytes(), np.uint8)
        rb = emb.shape[1] * 4
        kbs = [k.encode("utf-8") for k in keys]
        for kb in kbs:
            if not kb or b" " in kb or b"\0" in kb:
                raise ValueError(f"key must be non-empty without spaces: {kb!r}")
        klen = np.fromiter(map(len, kbs), dtype=np.int64, count=len(kbs))
        rec = klen + len(mid) + rb
        start = self._ark.tell() + np.concatenate([[0], np.cumsum(rec)[:-1]])
        # runs of equal-length keys (all of VoxCeleb's) are records of one size:
        # each run is laid out as one [run, record] byte matrix
        cut = np.flatnonzero(np.diff(klen)) + 1
        data = emb.view(np.uint8).reshape(len(kbs), rb)
        for a, b in zip(np.r_[0, cut], np.r_[cut, len(kbs)]):
            L = int(klen[a])
            m = np.empty((b - a, L + len(mid) + rb), np.uint8)
            m[:, :L] = np.frombuffer(b"".join(kbs[a:b]), np.uint8).reshape(b - a, L)
            m[:, L:L + len(mid)] = mid
            m[:, L + len(mid):] = data[a:b]
            self._ark.write(m.data)
        self._scp.write("".join(f"{k} {self.ark_path}:{o}\n"
                                for k, o in zip(keys, (start + klen + 1).tolist())))

    def close(self):
        if self._ark:
            self._ark.close()
            self._scp.close()
            self._ark = self._scp = None
            if self._atomic:
                os.replace(self.ark_path + self._sfx, self.ark_path)
                os.replace(self.scp_path + self._sfx, self.scp_path)

    def abort(self):
        """Close without publishing: an atomic writer deletes its temporary
        files, so a failed write never leaves a complete-looking pair."""
        if self._ark:
            self._ark.close()
            self._scp.close()
            self._ark = self._scp = None
            if self._atomic:
                for p in (self.ark_path + self._sfx, self.scp_path + self._sfx):
                    try:
                        os.remove(p)
                    except OSError:
                        pass

    def __enter__(self):
        return self

    def __exit__(self, exc_type, *a):
        if exc_type is not None and self._atomic:
            self.abort()
        else:
            self.close()


def read_vec_flt_ark(path):
    """Generator of (key, float32/float64 vector) over an FV/DV ark."""
    with open(path, "rb") as f:
        buf = f.read()
    pos = 0
    n = len(buf)
    while pos < n:
        key, pos = _read_key(buf, pos)
        if not key:
            break
        if buf[pos:pos + 2] != b"\0B":
            raise ValueError(f"{path}: only binary vectors are supported (key {key})")
        hdr = buf[pos + 2:pos + 5]
        if hdr == b"FV ":
            dt, es = np.float32, 4
        elif hdr == b"DV ":
            dt, es = np.float64, 8
        else:
            raise ValueError(f"{path}: unknown vector header {hdr!r}")
        dim = int(np.frombuffer(buf, np.int32, 1, pos + 6)[0])
        start = pos + 10
        yield key, np.frombuffer(buf, dt, dim, start).copy()
        pos = start + dim * es
