"""Weight blob: the build's stand-in for the reference's frozen GraphDef.

The reference ships a frozen TF1 `.pb` produced by `export_inference_model.sh`
(`tensorflow/export_inference_model.sh:30-44`) and loads it in
`tf_extract.py:75-82`.  Here the same variables travel as a flat, versioned
blob that both the native library (`csrc/blob.cpp`) and the CPU oracle read:

    b"VOXEMB01" | u64 header_len | header (ASCII) | pad to 64 | tensor data

The header is `key=value` lines describing the backbone (see `archs.py`),
then `tensors=N` and N lines `name|kind|d0,d1,...|offset|nbytes` (offsets are
relative to the data start, 64-byte aligned, little-endian float32).
Tensors are stored raw (HWIO kernels, BN moving statistics); BN folding and
kernel-native re-layout happen at load time in the library.
"""

from __future__ import annotations

import io
import struct

import numpy as np

from . import archs

MAGIC = b"VOXEMB01"
_LIST_KEYS = {"filters", "kernels", "dilations", "num_filters", "widths", "block_sizes",
              "block_strides", "k_sec", "inc_sec"}
_INT_KEYS = {"split", "output_dim", "expand_dim", "feat_dim", "num_init_features", "k_r",
             "bw", "cardinality"}


def _align(n, a=64):
    return (n + a - 1) // a * a


def spec_to_header(spec: dict) -> list:
    lines = []
    for k in sorted(spec):
        v = spec[k]
        if isinstance(v, (list, tuple)):
            v = ",".join(str(int(x)) for x in v)
        lines.append(f"{k}={v}")
    return lines


def header_to_spec(lines) -> dict:
    spec = {}
    for ln in lines:
        k, v = ln.split("=", 1)
        if k in _LIST_KEYS:
            spec[k] = [int(x) for x in v.split(",") if x]
        elif k in _INT_KEYS:
            spec[k] = int(v)
        else:
            spec[k] = v
    return spec


def save_blob(path_or_file, spec: dict, tensors: dict) -> None:
    """Write `tensors` (name -> float32 array) in manifest order."""
    man = archs.manifest(spec)
    entries, off = [], 0
    for name, shape, kind in man:
        if name not in tensors:
            raise KeyError(f"missing tensor {name}")
        a = np.ascontiguousarray(tensors[name], dtype=np.float32)
        if tuple(a.shape) != tuple(shape):
            raise ValueError(f"{name}: shape {a.shape} != manifest {shape}")
        entries.append((name, kind, shape, off, a.nbytes, a))
        off = _align(off + a.nbytes)
    lines = spec_to_header(spec) + [f"tensors={len(entries)}"]
    for name, kind, shape, o, nb, _ in entries:
        lines.append(f"{name}|{kind}|{','.join(str(d) for d in shape)}|{o}|{nb}")
    header = ("\n".join(lines) + "\n").encode("ascii")
    data_start = _align(len(MAGIC) + 8 + len(header))
    buf = io.BytesIO()
    buf.write(MAGIC)
    buf.write(struct.pack("<Q", len(header)))
    buf.write(header)
    buf.write(b"\0" * (data_start - buf.tell()))
    for name, kind, shape, o, nb, a in entries:
        pos = data_start + o
        buf.write(b"\0" * (pos - buf.tell()))
        buf.write(a.astype("<f4").tobytes())
    raw = buf.getvalue()
    if hasattr(path_or_file, "write"):
        path_or_file.write(raw)
    else:
        with open(path_or_file, "wb") as f:
            f.write(raw)


def load_blob(path_or_bytes):
    """Return (spec, ordered dict name -> float32 array) from a blob."""
    if isinstance(path_or_bytes, (bytes, bytearray, memoryview)):
        raw = bytes(path_or_bytes)
    else:
        with open(path_or_bytes, "rb") as f:
            raw = f.read()
    if raw[:8] != MAGIC:
        raise ValueError("not a VOXEMB01 weight blob")
    (hlen,) = struct.unpack("<Q", raw[8:16])
    lines = raw[16:16 + hlen].decode("ascii").strip().split("\n")
    data_start = _align(16 + hlen)
    ti = next(i for i, ln in enumerate(lines) if ln.startswith("tensors="))
    spec = header_to_spec(lines[:ti])
    n = int(lines[ti].split("=", 1)[1])
    tensors = {}
    for ln in lines[ti + 1:ti + 1 + n]:
        name, kind, dims, o, nb = ln.split("|")
        shape = tuple(int(d) for d in dims.split(",") if d)
        o, nb = int(o), int(nb)
        a = np.frombuffer(raw, dtype="<f4", count=nb // 4, offset=data_start + o)
        tensors[name] = a.reshape(shape).astype(np.float32)
    man = archs.manifest(spec)
    if [m[0] for m in man] != list(tensors):
        raise ValueError("blob tensor order does not match the backbone manifest")
    return spec, tensors
