"""`tf_extract.py` drop-in: FBANK scp in -> sliding CMN -> backbone -> FV ark+scp out.

Reference: tensorflow/tf_extract.py:45-113.  Same flags (--pb-file,
--expand-dim, --rspec <base> (reads <base>.scp), --wspec <base> (writes
<base>.ark/.scp)), same chunk rule (:96-111), same output bytes.  Differences,
all result-preserving:
  * chunks of equal length are batched together (the reference runs batch 1,
    :27); embeddings are batch-independent (bitwise, tests/test_gpu_parity.py);
  * no reader process / pickle queue: the shard is planned from the matrix
    headers, then each batch of chunks is decoded, CMN'd and sliced natively
    into a bounded ring of pinned buffers while earlier batches run on
    `--lanes` concurrent streams (stream.py);
  * --pb-file takes a VOXEMB01 weight blob (see weights.py / INTEGRATION.md);
  * an utterance shorter than 25 frames raises ZeroDivisionError, as the
    reference does at :111, before anything is written for later utterances.

    python -m voxsrc2020_speaker_verification_amd.extract --pb-file m.blob \\
        --expand-dim 3 --rspec data/voxceleb1/8-split/feats.1 --wspec out/xvector.1
"""

from __future__ import annotations

import argparse
import sys

import numpy as np

from .extractor import MIN_FRAMES, chunk_plan


def embed_utterances(feats, embed_batch, dim, batch=64, stack=np.stack):
    """feats: list of (key, [T,F] float32).  embed_batch(x[n,L,F]) -> [n,dim].
    Returns [len(feats), dim] float32 in input order, applying the chunk rule
    with chunks of equal length batched together.  `stack` builds a batch
    from the chunk slices (torch.stack for device-resident features)."""
    plans = []
    buckets = {}
    for u, (key, f) in enumerate(feats):
        plan = chunk_plan(f.shape[0])
        if not plan:
            raise ZeroDivisionError(f"utterance {key} has {f.shape[0]} < {MIN_FRAMES} frames "
                                    "(tf_extract.py:102,111)")
        plans.append(plan)
        for ci, (s, L) in enumerate(plan):
            buckets.setdefault(L, []).append((u, ci, s))
    chunk_emb = {}
    for L, items in buckets.items():
        for b in range(0, len(items), batch):
            part = items[b:b + batch]
            x = stack([feats[u][1][s:s + L] for (u, ci, s) in part])
            e = embed_batch(x)
            for (u, ci, s), row in zip(part, e):
                chunk_emb[(u, ci)] = row
    out = np.empty((len(feats), dim), np.float32)
    for u, plan in enumerate(plans):
        # target_values.append(value * length); sum(...) / sum(lengths) in float32
        acc = 0
        for ci, (s, L) in enumerate(plan):
            acc = acc + chunk_emb[(u, ci)] * L
        out[u] = acc / sum(L for _, L in plan)
    return out


def extract_scp(scp_path, embed_batch, dim, batch=64, cmn=True, threads=None):
    """(keys, embeddings) for every utterance of an scp, in scp order, through
    a synchronous embed function (host numpy in and out), streamed: headers
    first, then one batch of chunks at a time (stream.py)."""
    from .kaldi import read_scp
    from .stream import ChunkTable, SyncRunner, extract_stream
    table = ChunkTable(read_scp(scp_path), threads)
    keys, emb = extract_stream(table, lambda b: SyncRunner(table, embed_batch, cmn), batch)
    return keys, (emb if emb is not None else np.zeros((0, dim), np.float32))


def default_batch(extractor, batch):
    """batch <= 0: 256 chunks for a 1-D conv model (the TDNN: per-batch host
    work would otherwise rival its forward), 64 for the 2-D conv models."""
    return batch if batch > 0 else (256 if extractor.expand_dim == 2 else 64)


def open_lanes(pb_file, device, precision, lanes):
    """`lanes` extraction handles of one model on one device (stream.LanePool).
    lanes <= 0: automatic -- one lane for a 1-D conv model (the TDNN: its
    forward is so short that a second lane's launches only contend for the
    Python interpreter with the first's, profiles/r06g_extract_ragged_tdnn.json),
    four for the 2-D conv models (GPU-bound; extra lanes cover the host gaps)."""
    from .extractor import Extractor
    first = Extractor(pb_file, device=device, precision=precision)
    if lanes <= 0:
        lanes = 1 if first.expand_dim == 2 else 4
    return [first] + [Extractor(pb_file, device=device, precision=precision)
                      for _ in range(lanes - 1)]


def write_vectors(base, keys, emb, atomic=False):
    from .kaldi import VectorWriter
    with VectorWriter(base, atomic=atomic) as w:
        if len(keys):
            w.write_many(keys, np.asarray(emb, np.float32).reshape(len(keys), -1))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--pb-file", dest="pb_file", required=True,
                    help="VOXEMB01 weight blob (converted from the frozen .pb)")
    ap.add_argument("--expand-dim", dest="expand_dim", type=int, default=2,
                    help="2 for 1-D conv models (TDNN), 3 for 2-D conv models")
    ap.add_argument("--rspec", default="/tmp/fbank", help="fbank scp without '.scp'")
    ap.add_argument("--wspec", default="/tmp/xvector", help="output ark/scp base")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--batch", type=int, default=0,
                    help="chunks per batch (0: 256 for the TDNN, whose launches are short, "
                         "64 for the 2-D conv models)")
    ap.add_argument("--no-cmn", action="store_true", help="features are already CMN'd")
    ap.add_argument("--lanes", type=int, default=0,
                    help="concurrent extraction handles / streams per GPU (0: 1 for the TDNN, "
                         "4 for the 2-D conv models).  Each lane is a "
                         "full handle with its own copy of the weights and a workspace sized "
                         "for the largest batch (--batch x 1000 frames: ~5.6 GB for res2net50 at "
                         "--batch 64), so device memory grows with the lane count.  The lanes' "
                         "streams and pinned buffers come from PyTorch (ROCm build)")
    ap.add_argument("--reader-threads", type=int, default=None,
                    help="host threads decoding + CMN'ing features (default: usable CPUs, <= 16)")
    ap.add_argument("--device-reader", action="store_true",
                    help="decode the CM arks and apply the sliding CMN on the GPU (whole \"CM \" "
                         "matrices only; same bits as the host reader, about one host thread)")
    a = ap.parse_args(argv)
    import torch
    from .kaldi import read_scp
    from .stream import extract_entries
    torch.cuda.set_device(a.device)
    lanes = open_lanes(a.pb_file, a.device, a.precision, a.lanes)
    try:
        if lanes[0].expand_dim != a.expand_dim:
            print(f"warning: --expand-dim {a.expand_dim} but the model layout is "
                  f"{lanes[0].expand_dim}; using the model's", file=sys.stderr)
        keys, emb = extract_entries(read_scp(a.rspec + ".scp"), lanes,
                                    default_batch(lanes[0], a.batch),
                                    cmn=not a.no_cmn, threads=a.reader_threads,
                                    device_reader=a.device_reader or None)
    finally:
        for ex in lanes:
            ex.close()
    write_vectors(a.wspec, keys, emb)
    return 0


if __name__ == "__main__":
    sys.exit(main())
