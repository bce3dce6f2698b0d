"""Data-parallel extraction: one process per GPU + one RCCL gather to rank 0.

Reference: tensorflow/eval_inference_model.sh:27-40 starts `num_gpus`
independent tf_extract.py processes (CUDA_VISIBLE_DEVICES=i-1) on the
contiguous shards data/<set>/<N>-split/feats.<i>.scp and then "gathers" with
`cat xvector.{1..N}.ark > xvector.ark`.  Here each rank extracts the
split_scp.pl shard of the scp (or reads the reference's pre-split shard
file), then the per-rank embedding matrices are assembled on rank 0 with one
gather over RCCL/xGMI (backend "nccl"; "gloo" for CPU tests; `--all-gather`
delivers them to every rank instead).  Rank 0 writes the merged ark/scp in
shard order, i.e. byte-identical to the `cat`, plus (optionally) the cohort
speaker-mean matrix for AS-norm (snorm.py:45-67), formed without a
per-utterance Python step (scoring.speaker_means; tools/bench_cohort.py).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m \\
        voxsrc2020_speaker_verification_amd.dp_extract --pb-file m.blob \\
        --rspec data/voxceleb2_dev/fbank80 --wspec exp/emb/voxceleb2_dev/xvector \\
        --cohort-spk2utt data/voxceleb2_dev/spk2utt
"""

from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def gather_embeddings(keys, emb, group=None, device=None, dst=None):
    """Gather variable-sized [n_r, D] float32 matrices (+ their keys) from every
    rank, in rank order.  dst=None: all-gather, every rank returns (all_keys,
    [sum n_r, D]); dst=r: only rank r receives them (one RCCL gather of the
    matrices, the keys pickled to r alone) and the other ranks return
    ([], None) -- the merged ark and the cohort are rank 0's alone, so at
    VoxCeleb2-dev scale (1.09 M x 256 = 1.1 GB) nothing is copied to ranks
    that would drop it."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dim = emb.shape[1]
    dev = device if device is not None else torch.device("cpu")
    n = torch.tensor([emb.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    mx = max(counts)
    buf = torch.zeros((mx, dim), dtype=torch.float32, device=dev)
    if emb.shape[0]:
        buf[:emb.shape[0]] = torch.from_numpy(np.ascontiguousarray(emb)).to(dev)
    recv = dst is None or rank == dst
    if recv:
        # one receive slab, filled in rank order: no per-part host copies
        slab = torch.empty((world, mx, dim), dtype=torch.float32, device=dev)
        parts = list(slab.unbind(0))
    if dst is None:
        dist.all_gather(parts, buf, group=group)
        key_lists = [None] * world
        dist.all_gather_object(key_lists, list(keys), group=group)
    else:
        dist.gather(buf, parts if recv else None, dst=dst, group=group)
        key_lists = [None] * world if recv else None
        dist.gather_object(list(keys), key_lists, dst=dst, group=group)
    if not recv:
        return [], None
    host = slab.cpu().numpy()
    all_keys = [k for kl in key_lists for k in kl]
    if all(c == mx for c in counts):
        return all_keys, host.reshape(world * mx, dim)
    return all_keys, np.concatenate([host[r, :c] for r, c in enumerate(counts)], 0)


def rank_failures(failed, device=None, group=None):
    """All-gather one failure flag per rank; returns the failed rank ids."""
    import torch
    import torch.distributed as dist
    dev = device if device is not None else torch.device("cpu")
    flag = torch.tensor([1 if failed else 0], dtype=torch.int64, device=dev)
    flags = [torch.zeros_like(flag) for _ in range(dist.get_world_size(group))]
    dist.all_gather(flags, flag, group=group)
    return [r for r, f in enumerate(flags) if int(f.item())]


def run_tag(weights_path, precision):
    """What a shard's embeddings depend on besides its keys: the weight blob's
    bytes and the precision.  Stored beside each per-rank pair
    (`<wspec>.<i>.tag`) so --resume never reuses embeddings of another model."""
    import hashlib
    h = hashlib.sha256()
    with open(weights_path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 22), b""):
            h.update(blk)
    return f"sha256={h.hexdigest()} precision={precision}"


def _write_tag(base, tag):
    tmp = f"{base}.tag.part{os.getpid()}"
    with open(tmp, "w") as f:
        f.write(tag + "\n")
    os.replace(tmp, base + ".tag")


def completed_shard(wspec, rank, keys, dim, tag=None):
    """The embeddings of rank's shard if `<wspec>.<rank+1>.ark/.scp` already
    hold exactly `keys` (in order) as dim-D vectors -- and, when `tag` is given,
    were made by the same run tag (run_tag: weights + precision) -- else None.
    The pair is written atomically (VectorWriter(atomic=True)), so a shard
    interrupted mid-write is recomputed, never half-reused."""
    from .kaldi import read_vec_flt_ark
    base = f"{wspec}.{rank + 1}"
    if not (os.path.exists(base + ".ark") and os.path.exists(base + ".scp")):
        return None
    if tag is not None:
        try:
            with open(base + ".tag") as f:
                if f.read().strip() != tag:
                    return None
        except OSError:
            return None
    try:
        with open(base + ".scp") as f:
            if [ln.split()[0] for ln in f if ln.strip()] != list(keys):
                return None
        got = list(read_vec_flt_ark(base + ".ark"))
    except (OSError, ValueError, IndexError):
        return None
    if [k for k, _ in got] != list(keys) or any(np.shape(v) != (dim,) for _, v in got):
        return None
    return (np.stack([v for _, v in got]).astype(np.float32) if got
            else np.zeros((0, dim), np.float32))


def run(rank, world, scp_items, embed_fn, dim, wspec, shard_file=None, batch=64,
        device=None, write_per_rank=True, cohort_spk2utt=None, resume=False, shard_keys=None,
        tag=None, extract_shard=None, all_gather=False):
    """The per-rank body (also used by the gloo tests with a fake embedder).
    scp_items: full list of (key, feat) is NOT required -- each rank only
    decodes its own shard: `scp_items` is a callable(rank, world) -> list of
    (key, [T,F] features).  resume: a rank whose per-rank ark/scp already hold
    its shard (`shard_keys(rank, world)` -> keys, without decoding features)
    reuses them -- the reference's per-shard processes are restartable one by
    one in the same way (eval_inference_model.sh:29-36).  tag: the run tag
    (run_tag) written beside each per-rank pair and required to match on
    resume.  extract_shard: callable(rank, world) -> (keys, [n, dim]
    embeddings) that replaces scp_items + embed_fn (the CLI's streaming GPU
    pipeline, stream.extract_entries: the shard is never decoded whole).
    all_gather: every rank receives every embedding (returned everywhere);
    default False gathers to rank 0 only, the one rank that writes the merged
    ark and the cohort; the other ranks return ([], None)."""
    from .extract import embed_utterances, write_vectors
    err = None
    try:
        emb = None
        if resume and wspec and shard_keys is not None:
            keys = list(shard_keys(rank, world))
            emb = completed_shard(wspec, rank, keys, dim, tag)
        if emb is None:
            if extract_shard is not None:
                keys, emb = extract_shard(rank, world)
            else:
                feats = scp_items(rank, world)
                emb = (embed_utterances(feats, embed_fn, dim, batch) if feats
                       else np.zeros((0, dim), np.float32))
                keys = [k for k, _ in feats]
            if write_per_rank and wspec:
                # xvector.<i>.ark as the reference; atomic for --resume
                base = f"{wspec}.{rank + 1}"
                if tag is not None and os.path.exists(base + ".tag"):
                    os.remove(base + ".tag")     # stale until the new pair is in place
                write_vectors(base, keys, emb, atomic=True)
                if tag is not None:
                    _write_tag(base, tag)
    except Exception as e:   # e.g. ZeroDivisionError for a < 25-frame utterance
        err = e
    # every rank learns whether any shard failed BEFORE the gathers, so no rank
    # is left blocked in a collective (the reference's per-shard processes fail
    # independently, eval_inference_model.sh:29-36)
    failed = rank_failures(err is not None, device)
    if failed:
        if err is not None:
            raise err
        raise RuntimeError(f"extraction failed on rank(s) {failed}; rank {rank} aborts too")
    all_keys, all_emb = gather_embeddings(keys, emb, device=device,
                                          dst=None if all_gather else 0)
    if rank == 0 and wspec:
        write_vectors(wspec, all_keys, all_emb)           # == cat xvector.{1..N}.ark
        if cohort_spk2utt:
            from .scoring import read_spk2utt, speaker_means
            spk, cohort = speaker_means(all_keys, all_emb, read_spk2utt(cohort_spk2utt))
            np.save(wspec + ".cohort.npy", cohort.astype(np.float32, copy=False))
            with open(wspec + ".cohort.keys", "w") as f:
                f.write("\n".join(spk) + "\n")
    return all_keys, all_emb


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--pb-file", dest="pb_file", required=True)
    ap.add_argument("--rspec", required=True, help="<base> of <base>.scp (sharded here) or, "
                    "with --pre-split, the shard template '<dir>/feats' (feats.<i>.scp)")
    ap.add_argument("--pre-split", action="store_true")
    ap.add_argument("--wspec", required=True)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--batch", type=int, default=0,
                    help="chunks per batch (0: 256 for the TDNN, whose launches are short, "
                         "64 for the 2-D conv models)")
    ap.add_argument("--cohort-spk2utt", default=None)
    ap.add_argument("--lanes", type=int, default=0,
                    help="concurrent extraction handles / streams per GPU (0: 1 for the TDNN, "
                         "4 for the 2-D conv models; each its own "
                         "weights + a workspace for the largest batch: see extract --help)")
    ap.add_argument("--reader-threads", type=int, default=None)
    ap.add_argument("--device-reader", action="store_true",
                    help="decode + CMN on the GPU (see extract --help)")
    ap.add_argument("--resume", action="store_true",
                    help="reuse per-rank xvector.<i>.ark/.scp that already hold the rank's shard")
    ap.add_argument("--all-gather", action="store_true",
                    help="deliver every embedding to every rank (default: rank 0 only)")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", rank=rank, world_size=world,
                            device_id=torch.device("cuda", local))
    from .extract import default_batch, open_lanes
    from .kaldi import read_scp
    from .partition import shard
    from .stream import extract_entries

    def entries(r, w):
        if a.pre_split:
            return read_scp(f"{a.rspec}.{r + 1}.scp")
        return shard(read_scp(a.rspec + ".scp"), r, w)

    def keys(r, w):
        return [k for k, _ in entries(r, w)]

    lanes = open_lanes(a.pb_file, local, a.precision, a.lanes)
    batch = default_batch(lanes[0], a.batch)
    try:
        # the rank's shard streamed through its lanes (stream.py): planned from
        # the matrix headers, decoded one batch of chunks at a time
        run(rank, world, None, None, lanes[0].dim, a.wspec, batch=batch,
            device=torch.device("cuda", local), cohort_spk2utt=a.cohort_spk2utt,
            resume=a.resume, shard_keys=keys, tag=run_tag(a.pb_file, a.precision),
            extract_shard=lambda r, w: extract_entries(entries(r, w), lanes, batch,
                                                       threads=a.reader_threads,
                                                       device_reader=a.device_reader or None),
            all_gather=a.all_gather)
    finally:
        for ex in lanes:
            ex.close()
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
