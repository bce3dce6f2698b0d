"""Frozen TF1 GraphDef (.pb) -> VOXEMB01 weight blob.

The reference's boundary artefact is `<ckpt_dir>_<iter>.pb`, written by
`freeze_graph --output_node_names=outputs` (tensorflow/export_inference_model.sh:40-44)
from the graph of export_inference_graph.py:38-48.  Freezing turns every
variable into a `Const` node of the same name holding a TensorProto.  This
module walks the protobuf wire format directly (no TensorFlow, no .proto
files):

  GraphDef.node (1) -> NodeDef {name (1), op (2), input (3), attr (5): map<string, AttrValue>}
  AttrValue.tensor (8) -> TensorProto {dtype (1), tensor_shape (2), tensor_content (4),
                                       float_val (5, packed or not), double_val (6)}
  TensorShapeProto.dim (2) -> Dim {size (1)}
  AttrValue.f (4) -> float (FusedBatchNormV3 `epsilon`)

Tensors are matched to the backbone manifest (archs.manifest) by their TF
variable names; when names differ (a graph built under an extra scope), they
are matched in graph order by kind (kernel / moving_mean / moving_variance)
with shape checks.

    python -m voxsrc2020_speaker_verification_amd.pb2blob --pb-file m.pb \\
        --model-id res2net50_w24_s4_c32 --feat-dim 80 --out m.blob
"""

from __future__ import annotations

import argparse
import struct
import sys

import numpy as np

from . import archs, weights

DT_FLOAT, DT_DOUBLE = 1, 2


def _varint(buf, i):
    r = s = 0
    while True:
        b = buf[i]
        i += 1
        r |= (b & 0x7F) << s
        if not b & 0x80:
            return r, i
        s += 7


def fields(buf):
    """Yield (field_number, wire_type, value) of one protobuf message."""
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fn, wt, v


def parse_tensor(buf):
    dtype, shape, content = None, [], None
    fvals, dvals = [], []
    for fn, wt, v in fields(buf):
        if fn == 1:
            dtype = v
        elif fn == 2:
            for f2, _, d in fields(v):
                if f2 == 2:
                    size = 0
                    for f3, _, dv in fields(d):
                        if f3 == 1:
                            size = dv
                    shape.append(size)
        elif fn == 4:
            content = bytes(v)
        elif fn == 5:
            if wt == 2:
                fvals.extend(struct.unpack(f"<{len(v) // 4}f", v))
            else:
                fvals.append(struct.unpack("<f", v)[0])
        elif fn == 6:
            if wt == 2:
                dvals.extend(struct.unpack(f"<{len(v) // 8}d", v))
            else:
                dvals.append(struct.unpack("<d", v)[0])
    if dtype not in (DT_FLOAT, DT_DOUBLE):
        return None
    npdt = np.float32 if dtype == DT_FLOAT else np.float64
    count = int(np.prod(shape)) if shape else 1
    if content is not None:
        a = np.frombuffer(content, npdt).copy()
    else:
        vals = fvals if dtype == DT_FLOAT else dvals
        a = np.array(vals, npdt)
        if a.size == 1 and count > 1:           # TF stores splats as one value
            a = np.full(count, a[0], npdt)
    return a.reshape(shape).astype(np.float32)


def parse_graphdef(raw):
    """Returns (consts: ordered {name: array}, epsilons: [float] of FusedBatchNorm*)."""
    consts, eps = {}, []
    for fn, _, node in fields(raw):
        if fn != 1:
            continue
        name = op = None
        attrs = {}
        for f2, _, v in fields(node):
            if f2 == 1:
                name = bytes(v).decode()
            elif f2 == 2:
                op = bytes(v).decode()
            elif f2 == 5:
                k = val = None
                for f3, _, e in fields(v):
                    if f3 == 1:
                        k = bytes(e).decode()
                    elif f3 == 2:
                        val = e
                attrs[k] = val
        if op == "Const" and "value" in attrs:
            for f4, _, t in fields(attrs["value"]):
                if f4 == 8:
                    a = parse_tensor(t)
                    if a is not None:
                        consts[name] = a
        elif op and op.startswith("FusedBatchNorm") and "epsilon" in attrs:
            for f4, _, fv in fields(attrs["epsilon"]):
                if f4 == 4:
                    eps.append(struct.unpack("<f", fv)[0])
    return consts, eps


def _kind(name):
    for suf in ("/kernel", "/moving_mean", "/moving_variance"):
        if name.endswith(suf):
            return suf
    return None


def convert(raw, spec):
    consts, eps = parse_graphdef(raw)
    man = archs.manifest(spec)
    tensors = {}
    if all(n in consts for n, _, _ in man):
        for n, shape, _ in man:
            tensors[n] = consts[n]
    else:
        pools = {"/kernel": [], "/moving_mean": [], "/moving_variance": []}
        for n, a in consts.items():
            k = _kind(n)
            if k:
                pools[k].append((n, a))
        for n, shape, _ in man:
            k = _kind(n)
            if not pools[k]:
                raise ValueError(f"graph has too few {k} tensors for {spec['name']}")
            src, a = pools[k].pop(0)
            tensors[n] = a
        left = sum(len(v) for v in pools.values())
        if left:
            raise ValueError(f"graph has {left} unmatched variables for {spec['name']}")
    for n, shape, _ in man:
        if tuple(tensors[n].shape) != tuple(shape):
            raise ValueError(f"{n}: graph shape {tensors[n].shape} != expected {shape}")
    spec = dict(spec)
    if eps:
        spec["bn_eps_4d"] = repr(float(max(min(eps), 1.001e-5)))
    return spec, tensors


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--pb-file", required=True)
    ap.add_argument("--model-id", required=True, help=f"one of {sorted(archs.ARCHS)}")
    ap.add_argument("--feat-dim", type=int, default=80)
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    with open(a.pb_file, "rb") as f:
        raw = f.read()
    spec, tensors = convert(raw, archs.get_arch(a.model_id, a.feat_dim))
    weights.save_blob(a.out, spec, tensors)
    print(f"wrote {a.out}: {len(tensors)} tensors, "
          f"{archs.param_count(spec) / 1e6:.2f} M parameters", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
